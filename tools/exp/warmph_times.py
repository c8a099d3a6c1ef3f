"""Phase durations of k_bin_warm (variant `warmph`), averaged per workgroup, and the kernel span.
Usage: NR_LIB=tools/exp/warmph.so python tools/exp/warmph_times.py [config]"""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench
from libnativecpurenderer_amd import _lib
if os.environ.get("NR_LIB"):   # (tools only: the probe build instead of the shipped library)
    _lib.LIB_PATH = os.path.abspath(os.environ["NR_LIB"])
from libnativecpurenderer_amd import libNativeCPURendererPybind as R
cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]; xy, z, c = bench.make_scene(cfg)
ctx = R.RenderContext(cfg["W"], cfg["H"], False); buf = R.TriangleBuffer(xy, c, z=z, gouraud=cfg["gouraud"])
lib = _lib.load()
def frame():
    ctx.set_color(0, 0, 0, 0); ctx.set_depth_state(True, True); ctx.clear_depth(); ctx.draw_triangle_buffer(buf)
for _ in range(6): frame()
ctx.flush()
spans = []
acc_tot = np.zeros(8)
for _ in range(5):
    lib.ExpResetAcc()
    init = np.array([np.iinfo(np.uint64).max, 0], np.uint64)
    # reset span slots
    out = np.zeros(4 * 65536, np.uint64); out[0] = init[0]
    R.lib  # noqa
    lib.ExpSetTimes(out.ctypes.data_as(ctypes.c_void_p), 2)
    frame(); ctx.flush()
    acc = np.zeros(8, np.uint64); lib.ExpGetAcc(acc.ctypes.data_as(ctypes.c_void_p))
    lib.ExpGetItemTimes(out.ctypes.data_as(ctypes.c_void_p), 2)
    spans.append((int(out[1]) - int(out[0])) / 100.0)
    acc_tot += acc
n = acc_tot[7]
print("warm batches %d  " % ctx.warm_batch_count(), end="")
print("warm WGs/frame %d  per-WG us: loads %.2f  rects+LDS histogram %.2f  range reservation %.2f  pairs %.2f   kernel span %.2f us" % (
    n / 5, acc_tot[0] / n / 100, acc_tot[1] / n / 100, acc_tot[2] / n / 100, acc_tot[3] / n / 100, np.median(spans)))
