"""Warm binning (a TriangleBuffer drawn again under the binning key of its last
validated binning, k_bin_warm) against the CPU oracle, frame by frame, and its
checks: a warm batch whose binning fails (a tile over its kept range, pairs
missing, the binning's token never arriving) must still give the exact frame
(k_vis WarmCheck fallback) and latch the failure.

Geometry with off-screen clusters of huge-coordinate slivers: the cold count
bins a triangle with a screen coordinate beyond 1e7 into every column of its
rows (tri_tiles), so the warm binning's cluster cull must not drop such a
cluster by x.  Several frames per context, so every binning
set runs more than one epoch of its cursors."""
import numpy as np
import pytest

import scenes

pytestmark = pytest.mark.gpu


def _huge_cluster(rng, n=64):
    """64 triangles left of the screen (x in [-100, -50]); the first is a tall
    sliver spanning y = +-2e7 (binned full-width by the cold count)."""
    xy = np.empty((n, 6))
    for t in range(n):
        cx, cy = rng.uniform(-100, -50), rng.uniform(0, 400)
        xy[t] = [cx, cy, cx + 3, cy + 1, cx + 1, cy + 4]
    xy[0] = [-100.0, -2e7, -50.0, 2e7, -60.0, 0.0]
    z = rng.uniform(0, 1, size=(n, 3))
    c = rng.uniform(0, 1, size=(n, 12))
    c[:, 3::4] = 1.0
    return xy, z, c


def _scene(W, H, mesh_rc=(60, 200)):
    rng = np.random.default_rng(5)
    mesh = scenes.sphere_mesh(W, H, *mesh_rc)
    off1 = _huge_cluster(rng)
    off2 = _huge_cluster(rng)
    off2[0][:, 0::2] += W + 160.0   # right of the screen
    parts = [off1, mesh, off2]   # clusters of 64: the mesh starts at triangle 64
    pad = (-len(mesh[0])) % 64   # keep the second huge cluster aligned to a cluster boundary
    if pad:
        parts[1] = tuple(a[:len(a) - pad] for a in mesh)
    return tuple(np.ascontiguousarray(np.concatenate([p[k] for p in parts])) for k in range(3))


def _owned(H, n, r):
    from libnativecpurenderer_amd import sharding
    return sharding.owned_rows(H, n, r)


def _frames(fac, W, H, scene, nframes, shard=None, inject=None, hook=None):
    xy, z, c = scene
    ctx = fac.context(W, H, False)
    if fac.name == "gpu":
        from libnativecpurenderer_amd import libNativeCPURendererPybind as R
        ctx.set_warm_binning(1)
        if shard is not None:
            ctx.set_shard(*shard)
        buf = R.TriangleBuffer(xy, c, z=z, gouraud=True)
    outs, warm = [], []
    for k in range(nframes):
        if inject is not None and fac.name == "gpu" and k == inject[0]:
            ctx.set_warm_fault_injection(inject[1])
        if hook is not None and fac.name == "gpu":
            hook(k)
        ctx.set_color(0.1, 0.2, 0.3, 0.3 if k % 2 else 0.1)   # (non-uniform every other frame)
        ctx.set_depth_state(True, True)
        ctx.clear_depth()
        if fac.name == "gpu":
            ctx.draw_triangle_buffer(buf)
        else:
            ctx.draw_triangles(xy, c, z=z)
        outs.append({"f64": ctx.get_buffer_numpy(), "depth": ctx.get_depth_buffer()})
        if fac.name == "gpu":
            warm.append(ctx.warm_batch_count())
    ctx.warm_counts = warm
    return outs, ctx


@pytest.mark.parametrize("shard", [None, (2, 0), (2, 1), (8, 3)])
def test_warm_frames_with_huge_offscreen_clusters(gpu, oracle, shard):
    W, H = 640, 400
    scene = _scene(W, H)
    want, _ = _frames(oracle, W, H, scene, 8)
    got, ctx = _frames(gpu, W, H, scene, 8, shard=shard)
    rows = slice(None) if shard is None else _owned(H, *shard)
    for k, (g, o) in enumerate(zip(got, want)):
        assert scenes.bits_equal(g["f64"][rows], o["f64"][rows]), f"frame {k}: {scenes.first_mismatch(g['f64'][rows], o['f64'][rows])}"
        assert np.array_equal(g["depth"][rows], o["depth"][rows]), f"frame {k} depth"
    assert ctx.warm_batch_count() >= 5, ctx.warm_batch_count()   # frames 2..7 after the first validated draw
    assert ctx.warm_failure_count() == 0


@pytest.mark.parametrize("mode,mesh_rc", [(1, (60, 200)), (2, (60, 200)), (3, (60, 200)),
                                          (1, (250, 700)), (3, (250, 700))])
def test_warm_fault_falls_back_exactly(gpu, oracle, mode, mesh_rc):
    """A fault injected into the 4th frame's warm batch (1 ranges overflow, 2
    token withheld -- only on the beside-raster path of small batches, 3 a
    workgroup's pairs dropped; 350k triangles bin inline): every frame still
    equals the oracle's, the failure is counted and its message latched, and
    the next frames bin cold (1, 3: the buffer is banned from warm binning) or
    warm again after a new cold binning (2)."""
    from libnativecpurenderer_amd import _lib
    W, H = 640, 400
    scene = _scene(W, H, mesh_rc)
    want, _ = _frames(oracle, W, H, scene, 7)
    _lib.clear_error()
    got, ctx = _frames(gpu, W, H, scene, 7, inject=(3, mode))
    for k, (g, o) in enumerate(zip(got, want)):
        assert scenes.bits_equal(g["f64"], o["f64"]), f"frame {k}: {scenes.first_mismatch(g['f64'], o['f64'])}"
        assert np.array_equal(g["depth"], o["depth"]), f"frame {k} depth"
    assert ctx.warm_failure_count() == 1
    assert "warm binning" in _lib.last_error(), _lib.last_error()
    w = ctx.warm_counts   # batches binned warm after each frame
    assert w[3] > w[2], w  # the injected frame was a warm batch
    if mode == 2:
        assert w[6] > w[4], w   # warm again once a cold binning re-captured the schedule
    else:
        assert w[6] == w[3], w  # the buffer bins cold after a binning-check failure


def test_late_binning_is_ordered_before_main_stream_reuse(gpu, oracle):
    """a warm binning beside the raster that lands after the
    raster's token wait gave up (fault 4: the binning stream is held 1.5 s).
    The raster falls back (exact frame, one failure latched); the next batches
    bin cold on the main stream (the readbacks leave it idle) into the same
    binning sets and schedule the late binning writes -- they must wait for it
    (main_after_side_binning), so every frame still equals the oracle's."""
    from libnativecpurenderer_amd import _lib
    W, H = 640, 400
    scene = _scene(W, H)
    want, _ = _frames(oracle, W, H, scene, 9)
    _lib.clear_error()
    got, ctx = _frames(gpu, W, H, scene, 9, inject=(3, 4))
    for k, (g, o) in enumerate(zip(got, want)):
        assert scenes.bits_equal(g["f64"], o["f64"]), f"frame {k}: {scenes.first_mismatch(g['f64'], o['f64'])}"
        assert np.array_equal(g["depth"], o["depth"]), f"frame {k} depth"
    assert ctx.warm_failure_count() == 1
    assert "timed out" in _lib.last_error(), _lib.last_error()
    w = ctx.warm_counts
    assert w[8] > w[4], w   # warm again once a cold binning re-captured the schedule


def test_fresh_gate_set_beside_a_busy_device(gpu, oracle):
    """The token-word ordering of f1fb3a6 / ADVICE r05: a fresh context's
    first warm batches beside the raster (new binning sets, whose token words
    are zeroed on the binning stream) while the device is still busy with
    another context's long blended raster -- no raster may time out waiting
    for its token, and every frame is exact."""
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    busy = R.RenderContext(1920, 1080, False)
    bxy, bz, bc = scenes.triangle_soup(20000, 1920, 1080, 256, seed=9, alpha=(0.2, 0.8))
    bbuf = R.TriangleBuffer(bxy, bc, z=bz)
    busy.set_depth_state(True, False)

    def hook(k):   # before the fresh context's frames 1.. (its first warm ones): ~ms of ordered raster queued
        if k >= 1:
            busy.set_color(0, 0, 0, 0)
            for _ in range(4):
                busy.draw_triangle_buffer(bbuf)
    W, H = 640, 400
    scene = _scene(W, H)
    want, _ = _frames(oracle, W, H, scene, 6)
    got, ctx = _frames(gpu, W, H, scene, 6, hook=hook)
    for k, (g, o) in enumerate(zip(got, want)):
        assert scenes.bits_equal(g["f64"], o["f64"]), f"frame {k}"
        assert np.array_equal(g["depth"], o["depth"]), f"frame {k} depth"
    assert ctx.warm_failure_count() == 0
    assert ctx.warm_batch_count() >= 3
    busy.flush()


def _moving_frames(fac, W, H, scene, moves, shard=None, inject=None):
    """One frame per transform in `moves` ((tx, ty, deg) applied on top of
    the identity), the buffer drawn again every frame (GPU: TriangleBuffer)."""
    xy, z, c = scene
    ctx = fac.context(W, H, False)
    if fac.name == "gpu":
        from libnativecpurenderer_amd import libNativeCPURendererPybind as R
        ctx.set_warm_binning(1)
        if shard is not None:
            ctx.set_shard(*shard)
        buf = R.TriangleBuffer(xy, c, z=z, gouraud=True)
    outs, loose = [], []
    for k, (tx, ty, deg) in enumerate(moves):
        if inject is not None and fac.name == "gpu" and k == inject[0]:
            ctx.set_warm_fault_injection(inject[1])
        ctx.set_color(0.1, 0.2, 0.3, 0.1)
        ctx.set_depth_state(True, True)
        ctx.clear_depth()
        ctx.save_state()
        ctx.translate(tx, ty)
        if deg:
            ctx.rotate_degree(deg)
        if fac.name == "gpu":
            ctx.draw_triangle_buffer(buf)
        else:
            ctx.draw_triangles(xy, c, z=z)
        ctx.restore_state()
        outs.append({"f64": ctx.get_buffer_numpy(), "depth": ctx.get_depth_buffer()})
        if fac.name == "gpu":
            loose.append(ctx.loose_batch_count())
    ctx.loose_counts = loose
    return outs, ctx


# sub-pixel and pixel jitter, a rotation of a few hundredths of a degree (within 2 px at 640x400), a jump past
# 2 px (cold, a new schedule), then jitter around the new place
MOVES = [(0, 0, 0), (0.37, 0, 0), (0.9, -0.6, 0), (-1.4, 1.9, 0), (0.2, 0.1, 0.05), (1.99, -1.99, 0),
         (7.5, 3.0, 0), (7.9, 3.3, 0), (6.2, 2.0, 0), (0.0, 0.0, 0)]


@pytest.mark.parametrize("shard", [None, (2, 1), (8, 3)])
def test_loose_binning_of_a_moving_scene(gpu, oracle, shard):
    """A TriangleBuffer drawn under a new transform every frame (round 6):
    frames within 2 px of the last cold binning's transform bin into its
    loose ranges (k_bin_warm, k_vis slicing each tile's actual count), a jump
    beyond bins cold and becomes the new schedule.  Every frame equals the
    oracle's, bit for bit."""
    W, H = 640, 400
    scene = _scene(W, H)
    want, _ = _moving_frames(oracle, W, H, scene, MOVES)
    got, ctx = _moving_frames(gpu, W, H, scene, MOVES, shard=shard)
    rows = slice(None) if shard is None else _owned(H, *shard)
    for k, (g, o) in enumerate(zip(got, want)):
        assert scenes.bits_equal(g["f64"][rows], o["f64"][rows]), f"frame {k}: {scenes.first_mismatch(g['f64'][rows], o['f64'][rows])}"
        assert np.array_equal(g["depth"][rows], o["depth"][rows]), f"frame {k} depth"
    assert ctx.warm_failure_count() == 0
    # loose: frames 1-3 (within 2 px of frame 0), 7 and 8 (of frame 6); the rotated frame moves the huge
    # off-screen clusters by far more than 2 px, so frames 4-6 and 9 bin cold
    assert ctx.loose_counts == [0, 1, 2, 3, 3, 3, 3, 4, 5, 5], ctx.loose_counts


def test_loose_overflow_falls_back_exactly(gpu, oracle):
    """A loose batch whose tiles run past their loose ranges (fault 1 under a
    changed transform): those tiles are rasterised from every triangle (the
    frame stays exact), the failure is latched, and the buffer is not binned
    loose again (later moved frames bin cold, the exact repeat stays warm)."""
    from libnativecpurenderer_amd import _lib
    W, H = 640, 400
    scene = _scene(W, H)
    moves = [(0, 0, 0), (0.5, 0, 0), (0.25, 0.5, 0), (1.0, 1.0, 0), (0.5, 0.5, 0)]
    want, _ = _moving_frames(oracle, W, H, scene, moves)
    _lib.clear_error()
    got, ctx = _moving_frames(gpu, W, H, scene, moves, inject=(2, 1))
    for k, (g, o) in enumerate(zip(got, want)):
        assert scenes.bits_equal(g["f64"], o["f64"]), f"frame {k}: {scenes.first_mismatch(g['f64'], o['f64'])}"
        assert np.array_equal(g["depth"], o["depth"]), f"frame {k} depth"
    assert ctx.warm_failure_count() == 1
    assert "loose" in _lib.last_error(), _lib.last_error()
    assert ctx.loose_batch_count() == 2   # frames 1 and 2; none after the failure
