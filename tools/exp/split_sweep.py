"""Split-limit sweep (SetSplitLimits) of one bench configuration: the same
bench.py Runner, timed with each (split_at, dslice) pair, interleaved twice.
Usage: python tools/exp/split_sweep.py <config> "sa:ds,sa:ds,..." [emulate_shards]"""
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
import torch  # noqa: E402
torch.cuda.set_device(0)   # (torch first, as bench.py: the library is loaded after)
from libnativecpurenderer_amd import libNativeCPURendererPybind as R  # noqa: E402

cfg = sys.argv[1]
pairs = [tuple(int(v) for v in p.split(":")) for p in sys.argv[2].split(",")]
nsh = int(sys.argv[3]) if len(sys.argv) > 3 else 1
args = types.SimpleNamespace(no_kernel_timing=False, force_ordered=False, clock_settle_ms=60.0, root_slots="equal", frame_output="yuv420p",
                             emulate_shards=nsh)
R.set_device(0)
for rep in range(2):
    for sa, ds in pairs:
        run = bench.Runner(R, args, cfg, 1, 0, None, "cuda", nsh, 0)
        run.ctx.set_split_limits(sa, ds)
        r = run.run(20, 20)
        print(f"rep {rep} split_at {sa:5d} dslice {ds:5d}: {r['ms_per_step']:.4f} ms  k_vis {r['roofline']['kernel_us']} us",
              flush=True)
        del run
