"""Benchmark of the triangle raster hot path (BASELINE.json metric:
"Mpixels/s shaded+Z-tested (and fps) ... 1M tris; 1/2/4/8 GPU").

Workload: 3840x2160 RGB context, a 1,000,000-
triangle displaced UV sphere (synthetic, deterministic), Gouraud shading,
depth test LESS with write, both faces drawn.  One step = one frame:
uniform clear + depth clear + DrawTriangleBuffer of the whole mesh, with the
triangles already resident in HBM.  The work unit is a covered on-screen
pixel x triangle pair (counted once, outside the timed region, by the
library's fragment counter; equal to the oracle's count — tests check it).

Every step ends with the frame output: the u8 image (cpp:52-57, what the
video writer consumes) assembled on rank 0.  Multi-GPU (torchrun, one process
per GPU): the frame's 32-pixel tile rows are owned by the ranks in an
interleaved pattern; every rank bins and rasterises only its rows (no data-
path collective), then its rows of the u8 image go to rank 0 as one packed
RCCL message over xGMI, overlapped with the next frame.  Rank 0
also receives everyone's rows, so its share of the rows is calibrated before
the timed region (--root-slots auto: candidate weighted patterns timed, the
fastest kept and reported).  At N=1 the same step runs with a local conversion.
value = frame fragments (summed over ranks) x steps / max-over-ranks time.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

PEAK_HBM_GBPS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec

CONFIGS = {
    # name: (W, H, kind, params)
    "c3": dict(W=3840, H=2160, mesh=(500, 1000), gouraud=True, desc="C3: 1M-tri displaced UV sphere, 3840x2160, Gouraud, Z LESS+write"),
    "c3_1080p": dict(W=1920, H=1080, mesh=(500, 1000), gouraud=True, desc="1M-tri displaced UV sphere, 1920x1080, Gouraud, Z LESS+write"),
    "c2": dict(W=1920, H=1080, soup=(10000, 32.0, None), gouraud=False, desc="C2: 10k random opaque tris, 1920x1080, flat, Z LESS+write"),
    "c5": dict(W=1920, H=1080, soup=(50000, 256.0, (0.2, 0.8)), gouraud=False, write=False,
               desc="C5: 50k alpha-blended tris back-to-front, 1920x1080, Z test on, write off"),
}


def make_scene(cfg):
    import scenes
    if "mesh" in cfg:
        xy, z, c = scenes.sphere_mesh(cfg["W"], cfg["H"], *cfg["mesh"])
    else:
        n, spread, alpha = cfg["soup"]
        xy, z, c = scenes.triangle_soup(n, cfg["W"], cfg["H"], spread, seed=1234, alpha=alpha)
        if alpha is not None:   # back-to-front
            order = np.argsort(-z.mean(axis=1), kind="stable")
            xy, z, c = xy[order], z[order], c[order]
    return xy, z, c


FRAME_OUT_BPP = {"rgb": 3.0, "yuv420p": 1.5}   # frame output bytes per pixel (RGB context)


def algorithmic_bytes(cfg, n_tri, frac=1.0, u8=True, frame_out="rgb"):
    """B = N_tri*S_tri + W*H*(8*ipp + 4*[Z written]),
    S_tri = 104 B flat / 168 B Gouraud; ipp = 3 (RGB); plus the frame output
    every step hands over: the 3 B/pixel u8 image (GetBufferAsUInt8 /
    GatherFrameU8) or its 1.5 B/pixel YUV420P planes (--frame-output yuv420p).
    `frac`: the share of the frame one rank owns (tile-row shards)."""
    s_tri = 168 if cfg["gouraud"] else 104
    zw = 4 if cfg.get("write", True) else 0
    out = FRAME_OUT_BPP[frame_out] if u8 else 0.0
    return int(frac * (n_tri * s_tri + cfg["W"] * cfg["H"] * (8 * 3 + zw + out)))


EVENT_EVERY = 10   # timed-region frames per HIP-event-timed frame of the dominant kernel (each record pair
                   # perturbs the stream: 1 in 4 cost ~7 % of C3 throughput, 1 in 10 ~2 %)

KERNEL_SYMBOL = {"tile_raster": "k_vis (order-free) / k_tile_raster (ordered)"}


def kernel_bytes(cfg, n_tri, path, frac=1.0, frame_out="rgb"):
    """Algorithmic bytes of the dominant kernel per launch.
    Both rasterisers read each triangle (positions, depths, colours) once and
    write the framebuffer and depth once, all inside one kernel (k_vis shades
    its tiles itself; k_tile_raster keeps the tile in registers); k_vis also
    writes the u8 frame (k_to_u8_rows does it after the ordered raster)."""
    return {"tile_raster": algorithmic_bytes(cfg, n_tri, frac, u8=(path == "order-free"), frame_out=frame_out)}


def cpu_baseline(cfg, xy, z, c, budget_s=10.0, max_frames=50):
    """The oracle (CPU restatement, single thread) on the same frames."""
    import scenes
    f = scenes.OracleFactory()
    times, frags = [], 0
    ctx = f.context(cfg["W"], cfg["H"], False)
    t_start = time.perf_counter()
    while len(times) < max_frames and (time.perf_counter() - t_start < budget_s or len(times) < 2):
        t0 = time.perf_counter()
        ctx.set_color(0, 0, 0, 0)
        ctx.set_depth_state(True, cfg.get("write", True))
        ctx.clear_depth()
        ctx.draw_triangles(xy, c, z=z)
        times.append(time.perf_counter() - t0)
        frags = ctx.last_fragment_count()
    med = float(np.median(times))
    return {"value": frags / med / 1e6, "unit": "Mpixels/s", "cores": 1, "kind": "port",
            "sample": f"{len(times)} full frames of the same workload, median {med*1e3:.1f} ms/frame "
                      f"(oracle/oracle.c, gcc -O3 -ffp-contract=off, 1 thread)"}


def load_pmc_traffic(cfg_name):
    p = os.path.join(ROOT, "profiles", f"pmc_{cfg_name}.json")
    if os.path.exists(p):
        d = json.load(open(p))
        return d.get("hbm_bytes_per_launch"), d
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--extra", action="store_true", help="also time c2/c5 and report them under 'extra'")
    ap.add_argument("--no-kernel-timing", action="store_true", help="time without per-kernel HIP events")
    ap.add_argument("--force-ordered", action="store_true", help="A/B: always take the in-order tile raster")
    ap.add_argument("--emulate-shards", type=int, default=0,
                    help="experiment: render shard 0 of N on this one GPU (no gather) to time one rank's share")
    ap.add_argument("--gloo-test", action="store_true",
                    help="testing the N>1 orchestration on one GPU: gloo process group, CPU reductions, every rank "
                         "renders its shard on its LOCAL_RANK device but the RCCL frame gather is skipped")
    ap.add_argument("--frame-output", default="rgb", choices=sorted(FRAME_OUT_BPP),
                    help="frame output of every step: the u8 image (cpp:52-57) or its YUV420P planes (the video "
                         "encoder's input, PutRendererContextFrame cpp:232-275), written by the raster and gathered")
    ap.add_argument("--root-slots", default="auto",
                    help="N>1 (and --emulate-shards): tile-row share of rank 0, in bands per 2 bands of every other "
                         "rank (SetShardSlots); 'equal' = SetShard; 'auto' (N>1) times candidates and keeps the "
                         "fastest -- the root also receives every other rank's bands, so it gets less to render "
                         "when the gather dominates")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gloo_test:
        local_rank = 0   # every rank on the one GPU
    import torch
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.gloo_test:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    rdev = "cpu" if args.gloo_test else "cuda"   # device of the reduction tensors
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    R.set_device(local_rank)

    cfg = CONFIGS[args.config]
    W, H = cfg["W"], cfg["H"]
    xy, z, c = make_scene(cfg)
    n_tri = len(xy)
    ctx = R.RenderContext(W, H, False)
    ctx.set_frame_format(args.frame_output)
    if args.force_ordered:
        ctx.set_force_ordered_raster(True)
    buf = R.TriangleBuffer(xy, c, z=z, gouraud=cfg["gouraud"])
    comm = None
    nsh = world if world > 1 else max(1, args.emulate_shards)
    me = rank if world > 1 else 0

    def slots_for(k):
        return None if k is None else [k] + [2] * (nsh - 1)

    def apply_partition(k):
        if nsh <= 1:
            return
        if k is None:
            ctx.set_shard(nsh, me)
        else:
            ctx.set_shard_slots(nsh, me, slots_for(k))

    fixed_k = None if args.root_slots in ("auto", "equal") else int(args.root_slots)
    apply_partition(fixed_k)
    if world > 1 and not args.gloo_test:
        from libnativecpurenderer_amd import sharding
        comm = sharding.make_comm(dist, world, rank)

    def frame():
        ctx.set_color(0, 0, 0, 0)
        ctx.set_depth_state(True, cfg.get("write", True))
        ctx.clear_depth()
        ctx.draw_triangle_buffer(buf)
        ctx.gather_frame_u8(comm, 0)

    # fragment count of one frame (outside the timed region), summed over ranks
    ctx.set_fragment_counting(True)
    frame()
    ctx.flush()
    frags = ctx.get_fragment_count()
    ctx.set_fragment_counting(False)
    if dist is not None:
        t = torch.tensor([frags], dtype=torch.int64, device=rdev)
        dist.all_reduce(t)
        frags = int(t.item())

    def sync():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()

    # partition calibration (N>1, --root-slots auto): every candidate share of
    # rank 0 is timed over a few frames (max over ranks) and the fastest kept
    root_k, calib = fixed_k, {}
    if world > 1 and args.root_slots == "auto":
        for k in (None, 3, 4, 5, 6, 8, 10, 12):
            apply_partition(k)
            for _ in range(3):
                frame()
            ctx.flush()
            sync()
            t0 = time.perf_counter()
            for _ in range(10):
                frame()
            ctx.flush()
            torch.cuda.synchronize()
            t = torch.tensor([time.perf_counter() - t0], device=rdev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            calib["equal" if k is None else str(k)] = round(float(t.item()) / 10 * 1e3, 4)
        best = min(calib, key=calib.get)
        root_k = None if best == "equal" else int(best)
        apply_partition(root_k)

    for _ in range(args.warmup):
        frame()
    ctx.flush()

    names = ("tri_count", "tri_scan", "tri_emit", "tri_sort", "tile_ranges", "vis_init", "tile_raster",
             "resolve", "fill", "output", "gather")
    # (1) breakdown pass: HIP events around every kernel (they add ~50 us per
    #     frame of launch gaps, so this pass is not the headline)
    ctx.reset_kernel_timing()
    ctx.set_kernel_timing_filter("")
    ctx.enable_kernel_timing(True)
    for _ in range(args.steps):
        frame()
    ctx.flush()
    ctx.enable_kernel_timing(False)
    kernels = {}
    for name in names:
        tot, cnt = ctx.get_kernel_timing(name)
        if cnt:
            kernels[name] = round(tot / cnt * 1e3, 2)   # us per launch
    path = ctx.last_raster_path()
    from libnativecpurenderer_amd import sharding
    frac = len(sharding.owned_rows(H, nsh, me, slots=slots_for(root_k) if nsh > 1 else None)) / H
    kb = kernel_bytes(cfg, n_tri, path, frac, args.frame_output)
    dom = max((k for k in kb if k in kernels), key=lambda k: kernels[k])

    # (2) timed region: K frames, HIP events only around the dominant kernel
    #     (every EVENT_EVERY-th frame: each record leaves a few-us bubble on
    #     the stream, so sampling keeps the headline close to the untimed rate)
    ctx.reset_kernel_timing()
    ctx.set_kernel_timing_filter("" if args.no_kernel_timing else dom)
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        ctx.enable_kernel_timing(not args.no_kernel_timing and i % EVENT_EVERY == 0)
        frame()
    ctx.flush()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], device=rdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        dist.barrier()
    ctx.enable_kernel_timing(False)
    ms = dt / args.steps * 1e3
    tot, cnt = ctx.get_kernel_timing(dom)
    dom_us = round(tot / cnt * 1e3, 2) if cnt else kernels[dom]
    achieved = kb[dom] / (dom_us * 1e-6) / 1e9
    B = algorithmic_bytes(cfg, n_tri, frame_out=args.frame_output)   # whole job
    traffic, pmc = load_pmc_traffic(args.config)

    if rank != 0:
        return
    result = {
        "metric": "Mpixels/s shaded+Z-tested (and fps)",
        "value": round(frags * args.steps / dt / 1e6, 1),
        "unit": "Mpixels/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 4),
        "fps": round(1e3 / ms, 1),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (deterministic displaced UV sphere / seeded soup, SURVEY.md §8d)",
        "config": {"workload": cfg["desc"], "width": W, "height": H, "triangles": n_tri,
                   "fragments_per_frame": int(frags), "frame_pixels": W * H,
                   "frame_output": args.frame_output,
                   "parallelism": (f"tile-row shards x{world} + RCCL u8 frame gather" if world > 1
                                   else f"EMULATED shard 0 of {nsh} on one GPU (no gather)" if nsh > 1
                                   else "single GPU"),
                   **({"shard_slots": slots_for(root_k) or "equal", "partition_calibration_ms": calib}
                      if nsh > 1 else {})},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1),
                     "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                     "frac": round(achieved / PEAK_HBM_GBPS, 4),
                     "traffic": traffic,
                     "kernel": KERNEL_SYMBOL[dom], "kernel_us": dom_us,
                     "algorithmic_bytes_per_launch": kb[dom],
                     "frame_algorithmic_bytes": B,
                     "frame_achieved": round(B / (ms * 1e-3) / 1e9, 1),
                     "frame_frac": round(B / (ms * 1e-3) / 1e9 / PEAK_HBM_GBPS, 4)},
        "raster_path": path,
        "kernel_us": kernels,
        "kernel_us_note": f"per-launch averages from a breakdown pass with events around every kernel; the timed region records events around the dominant kernel on every {EVENT_EVERY}th frame (roofline.kernel_us)",
    }
    if not args.no_cpu_baseline and world == 1:
        result["cpu_baseline"] = cpu_baseline(cfg, xy, z, c)
        result["vs_cpu"] = round(result["value"] / result["cpu_baseline"]["value"], 1)
    print(json.dumps(result))


if __name__ == "__main__":
    main()
