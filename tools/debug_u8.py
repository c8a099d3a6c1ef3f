import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np, scenes
from libnativecpurenderer_amd import libNativeCPURendererPybind as R, _lib
g = scenes.GpuFactory()
def host_u8(f):
    t = f * 255
    ok = (t > -2147483649.0) & (t < 2147483648.0)
    return np.where(ok, np.trunc(np.where(ok, t, 0)).astype(np.int64) & 0xFF, 0).astype(np.uint8)
for name in ["shapes_rgba", "shapes_rgb", "shapes_rgba", "demo_t037", "shapes_rgba"]:
    out = scenes.run_scene(name, g)
    hu = host_u8(out["f64"])
    print(name, "u8==host(f64):", np.array_equal(hu, out["u8"]), "u8 sum", int(out["u8"].sum()), "err:", _lib.last_error())
ctx = R.RenderContext(80, 60, True)
ctx.set_color(0.5, 0.5, 0.5, 0.5)
ctx.draw_rect(1,1,5,5,1,0,0,1)
a = ctx.get_buffer_as_uint8_numpy(); print("simple 80x60 rgba u8 sum", int(a.sum()))
ctx.set_transform(0, 0, 0, 0, 0, 0)
ctx.draw_line(-1, -1, 1, 1, 2, 0.3, 0.3, 0.3, 0.5)
b = ctx.get_buffer_numpy(); a = ctx.get_buffer_as_uint8_numpy(); print("after singular line: f64 mean", b.mean(), "u8 sum", int(a.sum()), _lib.last_error())
