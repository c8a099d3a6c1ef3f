"""bench.py's roofline bookkeeping (CPU): the frame fraction of an emulated
rank share uses that share's bytes, a real N-GPU line N x the peak, and PMC
traffic is reported only from a summary of the same configuration and share."""
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_frame_fraction_uses_the_owned_share_and_n_peaks():
    b = _bench()
    B = b.algorithmic_bytes(b.CONFIGS["c3"], 1_000_000)
    assert B == 425_126_400
    # round-2 emulated 8-way share: 0.0527 ms per frame for ~1/8 of the rows
    r = b.frame_roofline(B, 270 / 2160, 0.0527, 1)
    assert r["frame_frac"] < 1 and r["frame_algorithmic_bytes"] == int(B * 270 / 2160)
    # a real 8-GPU line at the same per-frame time moves the whole frame over 8 GPUs
    r8 = b.frame_roofline(B, 270 / 2160, 0.0527, 8)
    assert r8["frame_peak"] == 8 * b.PEAK_HBM_GBPS and r8["frame_frac"] < 1
    assert abs(r8["frame_frac"] - r["frame_frac"]) < 1e-3   # an eighth of the bytes per GPU either way


def test_pmc_traffic_only_for_the_same_config_and_share(tmp_path, monkeypatch):
    b = _bench()
    monkeypatch.setattr(b, "ROOT", str(tmp_path))
    (tmp_path / "profiles").mkdir()
    (tmp_path / "profiles" / "pmc_c3.json").write_text(json.dumps({"config": "c3", "hbm_bytes_per_launch": 7}))
    assert b.load_pmc_traffic("c3")[0] == 7
    assert b.load_pmc_traffic("c3", 8)[0] is None                  # a rank share: no unsharded counters
    assert b.load_pmc_traffic("c2")[0] is None
    assert b.load_pmc_traffic("c3", frame_out="yuv420p")[0] is None
    tag = "c3" + b.shard_tag(8, [6, 2, 2, 2, 2, 2, 2, 2])
    (tmp_path / "profiles" / f"pmc_{tag}.json").write_text(json.dumps({"config": tag, "hbm_bytes_per_launch": 5}))
    assert b.load_pmc_traffic("c3", 8, [6, 2, 2, 2, 2, 2, 2, 2])[0] == 5
    assert b.load_pmc_traffic("c3", 8)[0] is None


def test_committed_pmc_summaries_name_their_config():
    """Every profiles/pmc_*.json says which configuration and share it measured
    (the file name's tag), so bench.py never applies one config's counters to another."""
    pdir = os.path.join(ROOT, "profiles")
    for f in os.listdir(pdir):
        if f.startswith("pmc_") and f.endswith(".json"):
            d = json.load(open(os.path.join(pdir, f)))
            assert d["config"] == f[len("pmc_"):-len(".json")], f
            assert d["hbm_bytes_per_launch"] > 0
