"""Per-work-item timeline of k_vis (probe build: NR_LIB=tools/exp/probe.so,
built with `make LIB=tools/exp/probe.so OBJ=/tmp/obj_probe EXTRA=-DNR_PROBE=1`).
Renders frames of a bench configuration (optionally one shard of N), clears
the probe before the last frame, and prints the schedule: kernel span, the
longest items, item duration by list length, and the busy workgroup count over
time.  Usage: NR_LIB=tools/exp/probe.so python tools/exp/probe_items.py [config] [shards]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
from libnativecpurenderer_amd import _lib  # noqa: E402
if os.environ.get("NR_LIB"):   # (tools only: the probe build instead of the shipped library)
    _lib.LIB_PATH = os.path.abspath(os.environ["NR_LIB"])
from libnativecpurenderer_amd import libNativeCPURendererPybind as R  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "c3"
shards = int(sys.argv[2]) if len(sys.argv) > 2 else 1
cfg = bench.CONFIGS[name]
xy, z, c = bench.make_scene(cfg)
ctx = R.RenderContext(cfg["W"], cfg["H"], False)
if shards > 1:
    ctx.set_shard(shards, 0)
buf = R.TriangleBuffer(xy, c, z=z, gouraud=cfg["gouraud"])
lib = _lib.load()
lib.NrProbeReset.restype = None
lib.NrProbeRead.restype = ctypes.c_long
lib.NrProbeRead.argtypes = [ctypes.c_void_p, ctypes.c_long]


def frame():
    ctx.set_color(0, 0, 0, 0)
    ctx.set_depth_state(True, cfg.get("write", True))
    ctx.clear_depth()
    ctx.draw_triangle_buffer(buf)


for _ in range(6):
    frame()
ctx.flush()
lib.NrProbeReset()
frame()
ctx.flush()
out = np.zeros(65536 * 8, np.uint64)
n = lib.NrProbeRead(out.ctypes.data, 65536)
e = out[: 8 * n].reshape(n, 8)
item = (e[:, 0] & 0xFFFFFFFF).astype(np.int64)
nt = (e[:, 0] >> 32).astype(np.int64)
tile = (e[:, 1] & 0xFFFFFFFF).astype(np.int64)
w = (e[:, 1] >> 32).astype(np.int64)
ls = (e[:, 2] & 0xFFFFFFFF).astype(np.int64)
le = (e[:, 2] >> 32).astype(np.int64)
dur = (e[:, 3] & 0xFFFFFF).astype(np.float64) / 100.0      # us (100 MHz)
t0 = (e[:, 3] >> 24).astype(np.float64) / 100.0
t0 -= t0.min()
t1 = t0 + dur
L = le - ls
nsl = w & 0xFFFF
print(f"{name} shards={shards}: {n} items, workgroup size {sorted(set(nt.tolist()))}, span {t1.max():.1f} us, "
      f"sum of item times {dur.sum():.0f} us (mean {dur.sum() / max(t1.max(), 1e-9):.0f} busy workgroups)")
print(f"split items (slices of dense tiles): {(nsl > 1).sum()}, empty tiles: {(L == 0).sum()}")
order = np.argsort(-t1)
print("last-finishing items (start, dur, end, tile, pairs, slices, item):")
for k in order[:12]:
    print(f"  {t0[k]:7.1f} {dur[k]:6.1f} {t1[k]:7.1f}  tile {tile[k]:5d}  {L[k]:5d} pairs  {nsl[k]} slices  item {item[k]}")
print("duration by list length (pairs: count, mean us, max us):")
for lo, hi in ((0, 1), (1, 64), (64, 128), (128, 256), (256, 512), (512, 768), (768, 1025), (1025, 1 << 30)):
    m = (L >= lo) & (L < hi)
    if m.any():
        print(f"  [{lo:5d},{hi:6d}) {m.sum():5d}  {dur[m].mean():6.1f}  {dur[m].max():6.1f}   split {(nsl[m] > 1).sum()}")
ts = np.linspace(0, t1.max(), 21)
busy = [int(((t0 <= t) & (t1 > t)).sum()) for t in ts]
print("busy workgroups over the span:", " ".join(str(b) for b in busy))
starts = np.sort(t0)
print("item starts at 25/50/75/90/100 %:", " ".join(f"{np.percentile(starts, p):.1f}" for p in (25, 50, 75, 90, 100)))

# phases (thread 0's clock at the barriers): keys set, raster done, merge done (split), hash done, records done, end
ph = np.stack([((e[:, 4] >> (16 * q)) & 0xFFFF) for q in range(4)] + [(e[:, 5] >> (16 * q)) & 0xFFFF for q in range(3)],
              1).astype(np.float64)
ph[ph == 0xFFFF] = np.nan
ph[ph == 0] = np.nan
ph /= 100.0
names = ["keys", "raster", "merge", "hash", "records", "w0data", "w0done"]
print("phase end times (us after item start), mean over items with pairs; single-slice / split-last:")
single = (L > 0) & (nsl == 1)
last = (L > 0) & (nsl > 1) & ~np.isnan(ph[:, 3])
for lab, m in (("single", single), ("split last", last)):
    if m.any():
        cols = [f"{nm} {np.nanmean(ph[m, q]):5.1f}" for q, nm in enumerate(names)]
        print(f"  {lab:10s} n={m.sum():5d}  " + "  ".join(cols) + f"  end {dur[m].mean():5.1f}")
