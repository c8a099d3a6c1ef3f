"""Round 6 probe: the driver-flag C3 line (the first measurement of a bench process) reads ~5-10 % slower
than the same workload measured later in the process (extra.c3_rgb, extra.c3_animated).  Runs the C3
Runner K times in one process (each a fresh Runner, as the extras are), 20 steps after 5 each, and prints
ms_per_step per run; optionally keeps the earlier Runners alive (as bench.py keeps the headline's).
Usage: [PROBE_PRE=alloc|ctx|run] python tools/exp/order_probe.py K [keep|drop] [clock settle ms]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    keep = len(sys.argv) > 2 and sys.argv[2] == "keep"
    settle = sys.argv[3] if len(sys.argv) > 3 else str(bench.CLOCK_SETTLE_MS)
    args = bench.parse_args(["--steps", "20", "--warmup", "5", "--no-cpu-baseline", "--no-extra",
                             "--clock-settle-ms", settle])
    if os.environ.get("PROBE_LIB"):   # a variant build (tools/exp/<name>.so)
        from libnativecpurenderer_amd import _lib
        _lib.LIB_PATH = os.path.abspath(os.environ["PROBE_LIB"])
    import torch
    torch.cuda.set_device(0)
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    R.set_device(0)
    alive = []
    pre = os.environ.get("PROBE_PRE", "")
    if pre == "alloc":   # 2 GB of device memory taken (and kept) before the first Runner
        alive.append(torch.empty(2 << 30, dtype=torch.uint8, device="cuda"))
    elif pre == "ctx":   # a throwaway 4K context drawn once and destroyed before the first Runner
        c = R.RenderContext(3840, 2160, False)
        c.set_color(0, 0, 0, 0)
        c.get_buffer_numpy()
        del c
    elif pre == "run":   # a throwaway C2 Runner first
        bench.Runner(R, args, "c2", 1, 0, None, "cuda", 1, 0, "none").run(args.steps, args.warmup)
    t0 = time.time()
    for i in range(k):
        run = bench.Runner(R, args, "c3", 1, 0, None, "cuda", 1, 0, "none")
        r = run.run(args.steps, args.warmup)
        print(f"run {i}: {r['ms_per_step']:.4f} ms/step  kernel_us {r['roofline']['kernel_us']}  "
              f"t={time.time() - t0:.1f}s verified={r.get('verified')}", flush=True)
        if keep:
            alive.append(run)
        else:
            del run


main()
