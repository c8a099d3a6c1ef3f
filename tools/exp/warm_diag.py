"""Warm-binning diagnostics for a bench configuration: N frames as bench.py's timed region draws them (no readback in
between), then the warm / failure counts and the latched error.  Usage: python tools/exp/warm_diag.py [config] [shards]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
from libnativecpurenderer_amd import libNativeCPURendererPybind as R, _lib  # noqa: E402
name = sys.argv[1] if len(sys.argv) > 1 else "c3"
shards = int(sys.argv[2]) if len(sys.argv) > 2 else 1
cfg = bench.CONFIGS[name]
xy, z, c = bench.make_scene(cfg)
ctx = R.RenderContext(cfg["W"], cfg["H"], False)
if shards > 1:
    ctx.set_shard(shards, 0)
buf = R.TriangleBuffer(xy, c, z=z, gouraud=cfg["gouraud"])
for rnd in range(3):
    _lib.clear_error()
    w0 = ctx.warm_batch_count()
    for i in range(30):
        ctx.set_color(0, 0, 0, 0); ctx.set_depth_state(True, True); ctx.clear_depth(); ctx.draw_triangle_buffer(buf)
        ctx.gather_frame_u8()
    ctx.flush()
    print(f"round {rnd}: warm {ctx.warm_batch_count() - w0}/30, failures {ctx.warm_failure_count()}, error: {_lib.last_error()!r}")
