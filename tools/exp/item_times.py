"""Per-work-item timeline of k_vis from the `times` variant (tools/exp):
renders C3 frames, reads the start/end clocks (s_memrealtime, 100 MHz) of
every work item of the last frame, and prints the schedule statistics."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
from libnativecpurenderer_amd import libNativeCPURendererPybind as R  # noqa: E402
from libnativecpurenderer_amd import _lib  # noqa: E402

cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
xy, z, c = bench.make_scene(cfg)
ctx = R.RenderContext(cfg["W"], cfg["H"], False)
if int(os.environ.get("ITEM_SHARDS", "1")) > 1:
    ctx.set_shard(int(os.environ["ITEM_SHARDS"]), 0)
buf = R.TriangleBuffer(xy, c, z=z)
for _ in range(4):
    ctx.set_color(0, 0, 0, 0)
    ctx.set_depth_state(True, True)
    ctx.clear_depth()
    ctx.draw_triangle_buffer(buf)
ctx.flush()
lib = _lib.load()
out = np.zeros(4 * 65536, np.uint64)
assert lib.ExpGetItemTimes(out.ctypes.data_as(ctypes.c_void_p), out.size) > 0
a = out.reshape(-1, 4)
a = a[a[:, 1] > a[:, 0]]
t0 = a[:, 0].astype(np.int64)
t1 = a[:, 1].astype(np.int64)
info = a[:, 2]
ntri = (info & 0xFFFFFFFF).astype(np.int64)
nsl = ((info >> 32) & 0xFFFF).astype(np.int64)
base = t0.min()
s, e = (t0 - base) / 100.0, (t1 - base) / 100.0   # us
dur = e - s
tm = (a[:, 3] & 0xFFFFFFFF).astype(np.int64)       # raster barrier, relative to the item start
tm2 = (a[:, 3] >> 32).astype(np.int64)             # split slices: after the merge
mid = np.where(tm > 0, s + tm / 100.0, e)
ras = mid - s          # item start -> raster barrier (key init + raster)
sha = e - mid          # shading (+ split-tile merge)
span = e.max()
print(f"items {len(a)}  span {span:.1f} us  sum(dur) {dur.sum():.0f} us  mean concurrency {dur.sum() / span:.0f}")
for lo, hi in ((0, 1), (1, 64), (64, 256), (256, 512), (512, 1025)):
    m = (ntri >= lo) & (ntri < hi) & (nsl <= 1)
    if m.any():
        print(f"  single tris [{lo},{hi}): n={m.sum():5d} dur mean {dur[m].mean():7.2f} max {dur[m].max():7.2f} us"
              f"  us/tri {dur[m].sum() / max(1, ntri[m].sum()):.4f}  raster {ras[m].mean():6.2f} shade {sha[m].mean():6.2f}")
m = nsl > 1
if m.any():
    print(f"  split slices: n={m.sum():5d} dur mean {dur[m].mean():7.2f} max {dur[m].max():7.2f} us"
          f"  us/tri {dur[m].sum() / max(1, ntri[m].sum()):.4f}  tris mean {ntri[m].mean():.0f}")
    after = np.where(tm2 > 0, tm2 / 100.0, dur)          # item start -> slot written + counter
    last = m & (e - (s + after) > 0.5)                   # the slices that went on to shade
    print(f"    raster {ras[m].mean():6.2f}  slot write+counter {(after[m] - ras[m]).mean():6.2f}"
          f"  last slices {last.sum()}: reduce+shade {(e[last] - s[last] - after[last]).mean() if last.any() else 0:6.2f}")
edges = np.arange(0, span + 2, 2.0)
act = np.zeros(len(edges))
for i, t in enumerate(edges):
    act[i] = ((s <= t) & (e > t)).sum()
order = np.argsort(-e)[:8]
print("last-finishing items (start, end, tris, slices):",
      "; ".join(f"{s[i]:.1f}-{e[i]:.1f} n={ntri[i]} sl={nsl[i]}" for i in order))
order = np.argsort(-dur)[:8]
print("longest items (start, end, tris, slices):",
      "; ".join(f"{s[i]:.1f}-{e[i]:.1f} n={ntri[i]} sl={nsl[i]}" for i in order))
print("active items every 2 us:", " ".join(str(int(x)) for x in act[::2]))
np.save(os.path.join(ROOT, "gpurun_out", "item_times.npy"), a)
