"""The frames bench.py times, checked against the oracle at full size
(VERDICT r05, next #1).

bench.Runner.frame is the timed step: clear + depth clear + DrawTriangleBuffer
of a resident TriangleBuffer + the frame output.  In the steady state it is
not the first frame of a context: it is the e-th warm epoch (e >= 2) of a
binning set (k_bin_warm into the kept schedule, beside the previous raster
behind k_gate_signal / k_gate_wait for >= 4 M-pixel shares, inline below), with
the fast clear leaving the empty tiles pending, and YUV420P planes written by
the raster.  These tests run that exact loop for 12 frames -- every binning
set through >= 3 warm epochs -- at C3 (1M triangles, 3840x2160), at the
metric's literal configuration (the same mesh at 1920x1080) and as 2- and
8-way tile-row shares of both, then read the last frame back and compare it
bit for bit with the oracle (f64 framebuffer, u32 depth, and the frame output
against scenes.yuv420p of the oracle's u8 image, or the u8 image itself), and
check bench.Runner.verify's digest verdict on the same frame.

Reference: the frame loop src/milrenderer.py:865-1038; blend cpp:515-549;
coverage cpp:822-845.
"""
import importlib.util
import os

import numpy as np
import pytest

import scenes

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FRAMES = 12


def _bench():
    spec = importlib.util.spec_from_file_location("bench_frames_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


_ORACLE = {}


def _oracle_frame(b, config, frame=0):
    """(f64, depth, u8) of one bench frame on the oracle (cached per config)."""
    key = (config, frame)
    if key not in _ORACLE:
        _ORACLE.clear()   # (one 4K frame held at a time: ~250 MB)
        cfg = b.CONFIGS[config]
        xy, z, c = b.make_scene(cfg)
        ctx = scenes.OracleFactory().context(cfg["W"], cfg["H"], False)
        ctx.set_color(0, 0, 0, 0)
        ctx.set_depth_state(True, cfg.get("write", True))
        ctx.clear_depth()
        if cfg.get("animate"):
            ctx.save_state()
            ctx.translate(b.anim_tx(frame), 0.0)
            ctx.draw_triangles(xy, c, z=z)
            ctx.restore_state()
        else:
            ctx.draw_triangles(xy, c, z=z)
        _ORACLE[key] = (ctx.get_buffer_numpy(), ctx.get_depth_buffer(), ctx.get_buffer_as_uint8_numpy(),
                        ctx.last_fragment_count())
    return _ORACLE[key]


def _run_frames(b, config, nsh, frame_output, nframes=FRAMES):
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    args = b.parse_args(["--emulate-shards", str(nsh), "--root-slots", "equal", "--frame-output", frame_output])
    run = b.Runner(R, args, config, 1, 0, None, "cpu", nsh, 0)
    for i in range(nframes):
        run.frame(i)
    run.drain()
    return run


def _owned_rows(b, H, nsh):
    from libnativecpurenderer_amd import sharding
    return sharding.owned_rows(H, nsh, 0) if nsh > 1 else np.arange(H)


def _yuv_rows(yuv, W, H, rows):
    """The Y rows `rows` and the chroma rows they own (even rows // 2) of flat planes."""
    cw, ch = W // 2, H // 2
    y = yuv[:W * H].reshape(H, W)
    u = yuv[W * H:W * H + cw * ch].reshape(ch, cw)
    v = yuv[W * H + cw * ch:].reshape(ch, cw)
    crow = rows[rows % 2 == 0] // 2
    return y[rows], u[crow], v[crow]


def _check(b, run, config, nsh):
    f64, depth, u8, frags = _oracle_frame(b, config)
    ctx, W, H = run.ctx, run.W, run.H
    rows = _owned_rows(b, H, nsh)
    assert ctx.warm_failure_count() == 0
    g = ctx.get_buffer_numpy()
    assert scenes.bits_equal(g[rows], f64[rows]), scenes.first_mismatch(g[rows], f64[rows])
    gd = ctx.get_depth_buffer()
    assert np.array_equal(gd[rows], depth[rows]), "depth"
    out = ctx.get_frame_u8()
    if run.frame_output == "yuv420p":
        want = scenes.yuv420p(u8)
        for k, (a, w) in enumerate(zip(_yuv_rows(out, W, H, rows), _yuv_rows(want, W, H, rows))):
            assert np.array_equal(a, w), f"plane {'YUV'[k]}: {np.argwhere(a != w)[:4]}"
    else:
        assert np.array_equal(out[rows], u8[rows]), np.argwhere(out[rows] != u8[rows])[:4]
    # bench.py's own check of the same frame against the committed oracle digests
    run.frags = frags
    ver = run.verify(FRAMES - 1)
    assert ver["verified"] is True, ver
    assert ver["warm_failures"] == 0


@pytest.mark.slow
@pytest.mark.parametrize("config", ["c3", "c3_1080p"])
@pytest.mark.parametrize("nsh", [1, 2, 8])
def test_bench_steady_state_frame_matches_oracle(gpu, config, nsh):
    b = _bench()
    run = _run_frames(b, config, nsh, "yuv420p")
    # frame 0 bins cold; from the frame after its validation every frame bins
    # warm, so each of the 3 binning sets runs >= 3 epochs of its cursors
    assert run.ctx.warm_batch_count() >= FRAMES - 3, run.ctx.warm_batch_count()
    _check(b, run, config, nsh)


@pytest.mark.slow
def test_bench_rgb_frame_output_matches_oracle(gpu):
    """extra.c3_rgb: the same loop with the u8 RGB image as the frame output."""
    b = _bench()
    run = _run_frames(b, "c3", 1, "rgb")
    _check(b, run, "c3", 1)


@pytest.mark.slow
def test_bench_animated_frames_match_oracle(gpu):
    """extra.c3_animated: a new sub-pixel translate every frame -- after the
    first cold binning, the frames bin into its loose ranges (the transform
    moves no vertex more than 2 px); the last frame of an 11- and a 12-frame
    run checked."""
    b = _bench()
    for nframes in (FRAMES, FRAMES - 1):
        run = _run_frames(b, "c3_animated", 1, "yuv420p", nframes)
        assert run.ctx.loose_batch_count() >= nframes - 3, run.ctx.loose_batch_count()
        f64, depth, u8, _ = _oracle_frame(b, "c3_animated", nframes - 1)
        g = run.ctx.get_buffer_numpy()
        assert scenes.bits_equal(g, f64), scenes.first_mismatch(g, f64)
        assert np.array_equal(run.ctx.get_depth_buffer(), depth)
        assert np.array_equal(run.ctx.get_frame_u8(), scenes.yuv420p(u8))
        ver = run.verify(nframes - 1)
        assert ver["verified"] is True and ver["warm_failures"] == 0, ver
        del run


@pytest.mark.slow
@pytest.mark.parametrize("config", ["c2", "c5"])
def test_bench_other_configs_match_oracle(gpu, config):
    """The extra lines' C2 (order-free, flat) and C5 (ordered blend) loops."""
    b = _bench()
    run = _run_frames(b, config, 1, "yuv420p", 6)
    f64, depth, u8, frags = _oracle_frame(b, config)
    g = run.ctx.get_buffer_numpy()
    assert scenes.bits_equal(g, f64), scenes.first_mismatch(g, f64)
    assert np.array_equal(run.ctx.get_depth_buffer(), depth)
    assert np.array_equal(run.ctx.get_frame_u8(), scenes.yuv420p(u8))
    run.frags = frags
    ver = run.verify(5)
    assert ver["verified"] is True, ver
