"""Phase durations of k_free_plan_r (variant `planr`): load, scan, items/classes, final stores, host stores."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench
from libnativecpurenderer_amd import libNativeCPURendererPybind as R, _lib
cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]; xy, z, c = bench.make_scene(cfg)
ctx = R.RenderContext(cfg["W"], cfg["H"], False); buf = R.TriangleBuffer(xy, c, z=z)
lib = _lib.load()
for _ in range(20):
    ctx.set_color(0, 0, 0, 0); ctx.set_depth_state(True, True); ctx.clear_depth(); ctx.draw_triangle_buffer(buf)
ctx.flush()
acc = np.zeros(8, np.uint64); lib.ExpGetAcc(acc.ctypes.data_as(ctypes.c_void_p))
n = int(min(acc[7], 4096))
out = np.zeros(8 * 4096, np.uint64); lib.ExpGetItemTimes(out.ctypes.data_as(ctypes.c_void_p), out.size)
a = out.reshape(-1, 8)[:n].astype(np.int64)
d = np.diff(a[:, :6], axis=1) / 100.0
print("plan_r calls", n, "T", a[0, 6], " phases (us, median): load %.2f  sums+classes %.2f  class scans+bases %.2f  offsets/items/stores %.2f  host stores %.2f" % tuple(np.median(d, 0)))
