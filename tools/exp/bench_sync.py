"""Frames with a host sync after each one (an application that reads every frame back before drawing the next):
clear + depth clear + DrawTriangleBuffer + Flush, timed over K frames.  Every batch is issued to an idle GPU, so
its binning cannot overlap a previous raster.  Usage: python tools/exp/bench_sync.py [config] [frames]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from libnativecpurenderer_amd import libNativeCPURendererPybind as R  # noqa: E402

cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 50
R.set_device(0)
xy, z, c = bench.make_scene(cfg)
ctx = R.RenderContext(cfg["W"], cfg["H"], False)
buf = R.TriangleBuffer(xy, c, z=z, gouraud=cfg["gouraud"])


def frame():
    ctx.set_color(0, 0, 0, 0)
    ctx.set_depth_state(True, cfg.get("write", True))
    ctx.clear_depth()
    ctx.draw_triangle_buffer(buf)
    ctx.flush()


for _ in range(5):
    frame()
ts = []
for _ in range(K):
    t0 = time.perf_counter()
    frame()
    ts.append(time.perf_counter() - t0)
ts.sort()
print(f"synced frames: median {ts[K // 2] * 1e3:.4f} ms, min {ts[0] * 1e3:.4f} ms over {K}")
