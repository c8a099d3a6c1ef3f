"""Reads the plan kernel's phase stamps (variant `plant`) after C3 frames."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench
from libnativecpurenderer_amd import libNativeCPURendererPybind as R, _lib
cfg = bench.CONFIGS["c3"]; xy, z, c = bench.make_scene(cfg)
ctx = R.RenderContext(cfg["W"], cfg["H"], False); buf = R.TriangleBuffer(xy, c, z=z)
lib = _lib.load(); out = np.zeros(8, np.uint64)
for i in range(6):
    ctx.set_color(0, 0, 0, 0); ctx.set_depth_state(True, True); ctx.clear_depth(); ctx.draw_triangle_buffer(buf); ctx.flush()
    lib.ExpGetItemTimes(out.ctypes.data_as(ctypes.c_void_p), 8)
    t = out.astype(np.int64)
    print("plan phases (us): pass1 %.2f pass2 %.2f host %.2f  ntiles %d" % ((t[1]-t[0])/100, (t[2]-t[1])/100, (t[3]-t[2])/100, t[4]))
