"""EXPERIMENT: would overlapping consecutive frames help?  K contexts (with
NR_CTX_STREAMS=1 each on its own stream) render frames of the same bench
configuration in turn; the frame period is compared with one context.
Usage: NR_CTX_STREAMS=1 python tools/exp/overlap_probe.py <config> <contexts> [shards]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
import torch  # noqa: E402
from libnativecpurenderer_amd import libNativeCPURendererPybind as R  # noqa: E402

name, K = sys.argv[1], int(sys.argv[2])
shards = int(sys.argv[3]) if len(sys.argv) > 3 else 1
torch.cuda.set_device(0)
R.set_device(0)
cfg = bench.CONFIGS[name]
xy, z, c = bench.make_scene(cfg)
buf = R.TriangleBuffer(xy, c, z=z, gouraud=cfg["gouraud"])
ctxs = []
for k in range(K):
    ctx = R.RenderContext(cfg["W"], cfg["H"], False)
    ctx.set_frame_format("yuv420p")
    if shards > 1:
        ctx.set_shard(shards, 0)
    ctxs.append(ctx)


def frame(i):
    ctx = ctxs[i % K]
    ctx.set_color(0, 0, 0, 0)
    ctx.set_depth_state(True, True)
    ctx.clear_depth()
    ctx.draw_triangle_buffer(buf)
    ctx.gather_frame_u8(None, 0)


for i in range(200):
    frame(i)
for cx in ctxs:
    cx.flush()
torch.cuda.synchronize()
for rep in range(3):
    n = 200
    t0 = time.perf_counter()
    for i in range(n):
        frame(i)
    for cx in ctxs:
        cx.flush()
    torch.cuda.synchronize()
    print(f"{name} shards={shards} contexts={K}: {(time.perf_counter() - t0) / n * 1e3:.4f} ms per frame", flush=True)
