"""C4 (BASELINE.json configs[3]) at its full size on one GPU: the 1M-triangle
4K C3 sphere rendered as 2, 4 and 8 tile-row shards (equal, and the weighted
root-heavy patterns `bench.py --root-slots` picks from), each shard in its own
context, then put back together two ways:

* the u8 frame output through GatherFrameU8's packed band assembly, with the
  packs moved by RCCL send/recv over a one-rank communicator
  (GatherFrameU8LocalRccl: the dlopen'd RCCL calls, group semantics and
  gather-stream ordering of the N-rank path) and by device copies
  (GatherFrameU8Local);
* the f64 framebuffer and the u32 depth buffer by bands on the host (each
  shard's owned 32-row bands, sharding.assemble).

Everything must equal the unsharded frame byte for byte, and the unsharded
frame itself equals the CPU oracle (the same check as test_c3_gouraud_depth_4k,
repeated here so the C4 assertion chain is self-contained).  The fragment
counts of the shards add up to the frame's.  What one GPU cannot cover is the
inter-process transport (xGMI links, the id exchange at N > 1 ranks).
"""
import numpy as np
import pytest

import scenes

pytestmark = [pytest.mark.gpu, pytest.mark.slow]

W, H = 3840, 2160


@pytest.fixture(scope="module")
def c3_scene():
    return scenes.sphere_mesh(W, H, 500, 1000)


def _frame(gpu, buf, n, r, slots):
    ctx = gpu.context(W, H, False)
    if n > 1:
        if slots is None:
            ctx.set_shard(n, r)
        else:
            ctx.set_shard_slots(n, r, slots)
    ctx.set_color(0, 0, 0, 0)
    ctx.set_depth_state(True, True)
    ctx.clear_depth()
    ctx.set_fragment_counting(True)
    ctx.draw_triangle_buffer(buf)
    ctx.flush()
    frags = ctx.get_fragment_count()
    ctx.set_fragment_counting(False)
    # a second, pipelined frame (binning stream, known sizes): the frame the
    # gather assembles is the steady-state one, not the counted first one
    ctx.set_color(0, 0, 0, 0)
    ctx.clear_depth()
    ctx.draw_triangle_buffer(buf)
    return ctx, frags


@pytest.fixture(scope="module")
def unsharded(gpu, oracle, c3_scene):
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    xy, z, c = c3_scene
    buf = R.TriangleBuffer(xy, c, z=z, gouraud=True)
    ctx, frags = _frame(gpu, buf, 1, 0, None)
    ctx.gather_frame_u8()
    full = {"f64": ctx.get_buffer_numpy(), "depth": ctx.get_depth_buffer(), "u8": ctx.get_frame_u8()}
    octx = oracle.context(W, H, False)
    octx.set_color(0, 0, 0, 0)
    octx.set_depth_state(True, True)
    octx.clear_depth()
    octx.draw_triangles(xy, c, z=z)
    assert scenes.bits_equal(full["f64"], octx.get_buffer_numpy()), "unsharded C3 f64 vs oracle"
    assert np.array_equal(full["depth"], octx.get_depth_buffer()), "unsharded C3 depth vs oracle"
    assert np.array_equal(full["u8"], octx.get_buffer_as_uint8_numpy()), "unsharded C3 u8 vs oracle"
    assert frags == octx.last_fragment_count()
    del ctx
    return buf, full, frags


def _root_slots(n, k):
    return None if k is None else [k] + [2] * (n - 1)


@pytest.mark.parametrize("n,root_k", [(2, None), (4, None), (8, None), (2, 3), (4, 5), (8, 6), (8, 12)])
def test_c4_shards_reassemble_to_the_c3_frame(gpu, unsharded, n, root_k):
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    from libnativecpurenderer_amd import sharding
    buf, full, full_frags = unsharded
    slots = _root_slots(n, root_k)
    ctxs, frags = [], 0
    for r in range(n):
        ctx, fr = _frame(gpu, buf, n, r, slots)
        assert ctx.get_shard_pattern() == sharding.band_pattern(n, slots)
        ctxs.append(ctx)
        frags += fr
    assert frags == full_frags

    # u8 frame: packed band gather through RCCL (one-rank communicator), root 0
    comm = R.Comm(1, 0, R.Comm.unique_id())
    R.RenderContext.gather_frame_u8_local_rccl(ctxs, comm, 0)
    got = ctxs[0].get_frame_u8()
    assert np.array_equal(got, full["u8"]), np.argwhere(got != full["u8"])[:5]
    # ... and through device copies, onto the last shard as root
    R.RenderContext.gather_frame_u8_local(ctxs, n - 1)
    got = ctxs[n - 1].get_frame_u8()
    assert np.array_equal(got, full["u8"]), np.argwhere(got != full["u8"])[:5]

    # f64 framebuffer and depth: owned bands of every shard, on the host
    fb = sharding.assemble([c.get_buffer_numpy() for c in ctxs], H, n, slots=slots)
    assert scenes.bits_equal(fb, full["f64"]), scenes.first_mismatch(fb, full["f64"])
    del fb
    dz = sharding.assemble([c.get_depth_buffer() for c in ctxs], H, n, slots=slots)
    assert np.array_equal(dz, full["depth"])
