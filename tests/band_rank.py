"""One rank of tests/test_band_delivery_gpu.py's two-process case: renders
shard `rank` of `nshards` of the test mesh and delivers its bands into the
shared host frame `name` (SharedHostBuffer), then exits.
Usage: python tests/band_rank.py NAME RANK NSHARDS FMT W H FRAMES"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def mesh(W, H):
    import scenes
    return scenes.sphere_mesh(W, H, 40, 90)


def render_frame(ctx, buf, k):
    ctx.set_color(0.05 * k, 0.1, 0.2, 0.3)
    ctx.set_depth_state(True, True)
    ctx.clear_depth()
    ctx.draw_triangle_buffer(buf)


def main():
    name, rank, nsh, fmt, W, H, frames = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4], \
        int(sys.argv[5]), int(sys.argv[6]), int(sys.argv[7])
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    xy, z, c = mesh(W, H)
    ctx = R.RenderContext(W, H, False)
    ctx.set_frame_format(fmt)
    ctx.set_shard(nsh, rank)
    buf = R.TriangleBuffer(xy, c, z=z, gouraud=True)
    nbytes = int(np.prod(ctx.frame_output_shape()))
    host = R.SharedHostBuffer(name, nbytes)
    t = None
    for k in range(frames):
        render_frame(ctx, buf, k)
        if t is not None:
            ctx.wait_frame_delivered(t)
        t = ctx.deliver_frame_bands(host)
    ctx.wait_frame_delivered(t)
    host.close()


if __name__ == "__main__":
    main()
