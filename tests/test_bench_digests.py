"""The oracle digests bench.py verifies its last timed frame against
(tests/golden/bench_digests.json, tests/golden/make_bench_digests.py) are the
oracle's: recomputed here on the CPU for the configurations the oracle renders
in about a second (the 1080p ones and one 4K frame of c3_animated), and every
entry has one digest per 32-row band of each buffer."""
import importlib.util
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_every_bench_config_has_complete_digests():
    b = _load("bench_dig", os.path.join(ROOT, "bench.py"))
    d = json.load(open(b.DIGEST_FILE))
    for name, cfg in b.CONFIGS.items():
        for fi in (b.ANIM_DIGEST_FRAMES if cfg.get("animate") else (0,)):
            e = d[b.digest_key(name, cfg, fi)]
            nb = (cfg["H"] + b.BAND_ROWS - 1) // b.BAND_ROWS
            assert (e["W"], e["H"], e["band_rows"]) == (cfg["W"], cfg["H"], b.BAND_ROWS)
            for kind in ("f64", "depth", "rgb", "yuv420p"):
                assert len(e[kind]) == nb and all(len(x) == 32 for x in e[kind]), (name, kind)


@pytest.mark.parametrize("config,frame", [("c3_1080p", 0), ("c2", 0), ("c3_animated", 19)])
def test_committed_digests_are_the_oracles(config, frame):
    b = _load("bench_dig2", os.path.join(ROOT, "bench.py"))
    g = _load("make_dig", os.path.join(ROOT, "tests", "golden", "make_bench_digests.py"))
    cfg = b.CONFIGS[config]
    xy, z, c = b.make_scene(cfg)
    f64, depth, u8, yuv, frags = g.oracle_frame(cfg, xy, z, c, b.anim_tx(frame) if cfg.get("animate") else 0.0)
    want = json.load(open(b.DIGEST_FILE))[b.digest_key(config, cfg, frame)]
    got = g.band_digests(b, f64, depth, u8, yuv, cfg["W"], cfg["H"])
    assert frags == want["fragments"]
    for kind in got:
        assert got[kind] == want[kind], kind
