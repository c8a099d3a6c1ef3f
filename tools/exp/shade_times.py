"""Shading phase durations (variant `sht`): hash / records / pixels, averaged over the shade_tile calls of C3 frames."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench
from libnativecpurenderer_amd import libNativeCPURendererPybind as R, _lib
cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]; xy, z, c = bench.make_scene(cfg)
ctx = R.RenderContext(cfg["W"], cfg["H"], False); buf = R.TriangleBuffer(xy, c, z=z)
lib = _lib.load(); out = np.zeros(8, np.uint64)
def frame():
    ctx.set_color(0, 0, 0, 0); ctx.set_depth_state(True, True); ctx.clear_depth(); ctx.draw_triangle_buffer(buf)
for _ in range(3): frame()
ctx.flush(); lib.ExpResetAcc()
for _ in range(5): frame()
ctx.flush(); lib.ExpGetAcc(out.ctypes.data_as(ctypes.c_void_p))
n = max(1, int(out[3]))
print("shade_tile calls %d  winners/tile %.1f  hash %.2f us  records %.2f us  pixels %.2f us  overflow pixels %.2f us" % (
    n, out[4] / n, out[0] / n / 100, out[1] / n / 100, out[2] / n / 100, out[5] / n / 100))
