"""Ingress-free frame assembly (DeliverFrameBands, §8e): every shard of a
frame copies its own bands of the frame output straight into their places in
one host frame -- no GPU receives the others' bands.  The assembled host frame
must equal the unsharded frame's output byte for byte: equal and weighted
band patterns, u8 RGB and YUV420P output, frame heights that end in a short
band, several frames in flight (two frame buffers, tickets); and across two
processes through POSIX shared memory (SharedHostBuffer), as one process per
GPU runs it."""
import os
import subprocess
import sys

import numpy as np
import pytest

import band_rank

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _reference(R, W, H, fmt, k):
    xy, z, c = band_rank.mesh(W, H)
    ctx = R.RenderContext(W, H, False)
    ctx.set_frame_format(fmt)
    buf = R.TriangleBuffer(xy, c, z=z, gouraud=True)
    band_rank.render_frame(ctx, buf, k)
    ctx.gather_frame_u8()
    return ctx.get_frame_u8().ravel().copy()


@pytest.mark.parametrize("fmt", ["rgb", "yuv420p"])
@pytest.mark.parametrize("W,H,part", [(320, 256, ("equal", 2)), (330, 330, ("equal", 3)),
                                      (256, 270, ("slots", [3, 1, 2])), (200, 100, ("equal", 1)),
                                      (2048, 2016, ("equal", 2))])   # (> 3 MB per rank: the strided copies)
def test_bands_assemble_the_frame(fmt, W, H, part):
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    xy, z, c = band_rank.mesh(W, H)
    kind, arg = part
    n = arg if kind == "equal" else len(arg)
    ctxs, bufs = [], []
    for r in range(n):
        ctx = R.RenderContext(W, H, False)
        ctx.set_frame_format(fmt)
        if kind == "equal":
            ctx.set_shard(n, r)
        else:
            ctx.set_shard_slots(n, r, arg)
        ctxs.append(ctx)
        bufs.append(R.TriangleBuffer(xy, c, z=z, gouraud=True))
    nbytes = int(np.prod(ctxs[0].frame_output_shape()))
    hosts = [R.HostBuffer(nbytes), R.HostBuffer(nbytes)]
    pending = {}
    for k in range(4):   # frame k into host frame k % 2; frame k - 2's copies waited on first
        h = hosts[k % 2]
        for r, ctx in enumerate(ctxs):
            if (k - 2, r) in pending:
                ctx.wait_frame_delivered(pending.pop((k - 2, r)))
        if k >= 2:
            got = h.array()[:nbytes].copy()
            want = _reference(R, W, H, fmt, k - 2)
            assert np.array_equal(got, want), f"frame {k - 2}: {np.count_nonzero(got != want)} bytes differ"
        h.array()[:] = 0xA5   # (every byte must be rewritten by some rank)
        for r, ctx in enumerate(ctxs):
            band_rank.render_frame(ctx, bufs[r], k)
            pending[(k, r)] = ctx.deliver_frame_bands(h)
    for (k, r), t in sorted(pending.items()):
        ctxs[r].wait_frame_delivered(t)
    for k in (2, 3):
        assert np.array_equal(hosts[k % 2].array()[:nbytes], _reference(R, W, H, fmt, k)), f"frame {k}"


@pytest.mark.parametrize("fmt", ["yuv420p"])
def test_two_processes_assemble_one_shared_host_frame(fmt):
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    W, H, frames, n = 384, 288, 3, 2
    name = f"/nr_band_test_{os.getpid()}"
    probe = R.RenderContext(W, H, False)
    probe.set_frame_format(fmt)
    nbytes = int(np.prod(probe.frame_output_shape()))
    del probe
    host = R.SharedHostBuffer(name, nbytes, owner=True)
    try:
        host.array()[:] = 0xA5
        procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "band_rank.py"), name, str(r), str(n), fmt,
                                   str(W), str(H), str(frames)]) for r in range(n)]
        for p in procs:
            assert p.wait(timeout=110) == 0
        want = _reference(R, W, H, fmt, frames - 1)
        got = host.array()[:nbytes]
        assert np.array_equal(got, want), f"{np.count_nonzero(got != want)} bytes differ"
    finally:
        host.close()


class _Pageable:
    """A plain numpy array as the host frame (not pinned: no device address)."""
    def __init__(self, nbytes):
        self.buf = np.full(nbytes, 0xA5, dtype=np.uint8)
        self.ptr, self.nbytes = self.buf.ctypes.data, nbytes


@pytest.mark.parametrize("fmt", ["rgb", "yuv420p"])
def test_bands_into_pageable_host_memory(fmt):
    """A host frame that is not pinned: the copy kernel cannot
    write through a device address, so the runtime copies take the share --
    the frame is still assembled exactly, and no error is latched."""
    from libnativecpurenderer_amd import _lib
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    W, H, n = 320, 256, 2
    xy, z, c = band_rank.mesh(W, H)
    _lib.clear_error()
    ctxs = []
    for r in range(n):
        ctx = R.RenderContext(W, H, False)
        ctx.set_frame_format(fmt)
        ctx.set_shard(n, r)
        ctxs.append((ctx, R.TriangleBuffer(xy, c, z=z, gouraud=True)))
    host = _Pageable(int(np.prod(ctxs[0][0].frame_output_shape())))
    for ctx, buf in ctxs:
        band_rank.render_frame(ctx, buf, 0)
        ctx.wait_frame_delivered(ctx.deliver_frame_bands(host))
    assert np.array_equal(host.buf, _reference(R, W, H, fmt, 0))
    assert _lib.last_error() == "", _lib.last_error()
