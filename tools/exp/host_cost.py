"""Host-side cost per frame of the bench's frame() sequence on a tiny scene
(the GPU work is negligible, so the loop rate is the submission rate), with a
per-call breakdown.  Usage: python tools/exp/host_cost.py [shards]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import scenes  # noqa: E402
from libnativecpurenderer_amd import libNativeCPURendererPybind as R  # noqa: E402

W, H = 256, 256
xy, z, c = scenes.triangle_soup(64, W, H, 10, seed=3, gouraud=True)
ctx = R.RenderContext(W, H, False)
sh = int(sys.argv[1]) if len(sys.argv) > 1 else 1
if sh > 1:
    ctx.set_shard(sh, 0)
buf = R.TriangleBuffer(xy, c, z=z)
calls = {"set_color": lambda: ctx.set_color(0, 0, 0, 0),
         "set_depth_state": lambda: ctx.set_depth_state(True, True),
         "clear_depth": lambda: ctx.clear_depth(),
         "draw_triangle_buffer": lambda: ctx.draw_triangle_buffer(buf),
         "gather_frame_u8": lambda: ctx.gather_frame_u8(None, 0)}
for _ in range(50):
    for f in calls.values():
        f()
ctx.flush()
N = 2000
tot = {k: 0.0 for k in calls}
t0 = time.perf_counter()
for _ in range(N):
    for k, f in calls.items():
        a = time.perf_counter()
        f()
        tot[k] += time.perf_counter() - a
ctx.flush()
dt = time.perf_counter() - t0
print(f"frame loop: {dt / N * 1e6:.1f} us/frame (shards={sh})")
for k, v in tot.items():
    print(f"  {k:22s} {v / N * 1e6:7.2f} us")
