"""Benchmark of the triangle raster hot path (BASELINE.json metric:
"Mpixels/s shaded+Z-tested (and fps) ... 1M tris; 1/2/4/8 GPU").

Workload: 3840x2160 RGB context, a 1,000,000-
triangle displaced UV sphere (synthetic, deterministic), Gouraud shading,
depth test LESS with write, both faces drawn.  One step = one frame:
uniform clear + depth clear + DrawTriangleBuffer of the whole mesh, with the
triangles already resident in HBM.  The work unit is a covered on-screen
pixel x triangle pair (counted once, outside the timed region, by the
library's fragment counter; equal to the oracle's count — tests check it).

Every step ends with the frame output: the frame's YUV420P planes (what the
video writer's encoder consumes, PutRendererContextFrame cpp:232-275; the u8
RGB image of cpp:52-57 with --frame-output rgb) assembled on rank 0.
Multi-GPU (torchrun, one process per GPU): the frame's 32-pixel tile rows are
owned by the ranks in an interleaved pattern; every rank bins and rasterises
only its rows (no data-path collective), then its rows of the frame output go
to rank 0 as one packed
RCCL message over xGMI, overlapped with the next frame.  Rank 0
also receives everyone's rows, so its share of the rows is calibrated before
the timed region (--root-slots auto: candidate weighted patterns timed, the
fastest kept and reported).  At N=1 the same step runs with a local conversion.
value = frame fragments (summed over ranks) x steps / max-over-ranks time.

At N=1 the line also carries `extra`: the metric's literal configuration
(1M triangles at 1920x1080), C2, C5 (with a VALU roofline beside the HBM one)
and host-delivered frame rates (--deliver host: every step ends with the
frame on the host, as the video caller needs it), each measured the same way.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

PEAK_HBM_GBPS = 8000.0   # MI355X_MICROARCH.md: 8.0 TB/s spec
# f64 VALU: 256 CUs x 4 SIMDs x 16 f64 lanes per clock x 2.4 GHz (78.6 TFLOP/s FP64 vector spec = this x 2 for FMA);
# a non-FMA f64 add or multiply counts one op
PEAK_F64_VALU_TOPS = 256 * 4 * 16 * 2.4e9 / 1e12

CONFIGS = {
    # name: (W, H, kind, params)
    "c3": dict(W=3840, H=2160, mesh=(500, 1000), gouraud=True, desc="C3: 1M-tri displaced UV sphere, 3840x2160, Gouraud, Z LESS+write"),
    "c3_1080p": dict(W=1920, H=1080, mesh=(500, 1000), gouraud=True, desc="1M-tri displaced UV sphere, 1920x1080, Gouraud, Z LESS+write (the metric's literal configuration)"),
    "c3_animated": dict(W=3840, H=2160, mesh=(500, 1000), gouraud=True, animate=True,
                        desc="C3 with a different transform every frame (translate anim_tx(i) = 0.005 + 0.01 (i % 100) "
                             "px, as milrenderer.py:980-1010 re-transforms every note every frame): no frame repeats "
                             "the binning key of another within 100 frames; frames within 2 px of the last cold "
                             "binning's transform bin into its loose ranges"),
    "c2": dict(W=1920, H=1080, soup=(10000, 32.0, None), gouraud=False, desc="C2: 10k random opaque tris, 1920x1080, flat, Z LESS+write"),
    "c5": dict(W=1920, H=1080, soup=(50000, 256.0, (0.2, 0.8)), gouraud=False, write=False,
               desc="C5: 50k alpha-blended tris back-to-front, 1920x1080, Z test on, write off"),
}

# f64 VALU operations a blended RGB fragment needs at least: per channel
# dst*(1-a) + (src*a), with (1-a) and src*a formed once per flat triangle --
# one multiply and one add (ApplyPixel, cpp:529-547); the depth test of C5 is
# provably passed per triangle, so it adds none
BLEND_OPS_PER_FRAGMENT = 6


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


# untimed frames before the warmup steps until the GPU has been under load this
# long: its clocks ramp for ~30 ms after idle, so a short run (the driver's
# --warmup 5 --steps 20) would otherwise time part of the ramp (~3-6 %,
# profiles/r04/warmup_steps20.txt).  Reported as "clock_settle" in the line.
# Round 6: 250 ms -- the C3 line at the driver's flags read 0.1293 ms (mean of 3)
# after 60 ms and 0.1252 after 250 ms on the same box, each rep lower; 1000 ms no
# better (profiles/r06/ab_settle.txt).
CLOCK_SETTLE_MS = 250.0

KERNEL_SYMBOL = {"tile_raster": "k_vis (order-free) / k_tile_raster (ordered)"}


def kernel_bytes(cfg, n_tri, path, frac=1.0, frame_out="rgb"):
    """Algorithmic bytes per launch of the path's kernels.
    The tiled rasterisers read each triangle (positions, depths, colours) once
    and write the framebuffer and depth once, all inside one kernel (k_vis
    shades its tiles itself; k_tile_raster keeps the tile in registers); k_vis
    also writes the u8 frame (k_to_u8_rows does it after the ordered raster)."""
    return {"tile_raster": algorithmic_bytes(cfg, n_tri, frac, u8=(path == "order-free"), frame_out=frame_out)}


def frame_roofline(B_frame, share, ms, world):
    """Frame-level HBM fraction.  A real N-GPU line moves the whole job's bytes
    with N GPUs' bandwidth; an emulated rank share (world 1, share < 1) moves
    its owned share of the bytes with one GPU's."""
    nbytes = B_frame if world > 1 else B_frame * share
    peak = PEAK_HBM_GBPS * max(1, world)
    achieved = nbytes / (ms * 1e-3) / 1e9
    return {"frame_algorithmic_bytes": int(nbytes), "frame_achieved": round(achieved, 1),
            "frame_peak": peak, "frame_frac": round(achieved / peak, 4)}


def shard_tag(nsh, slots):
    if nsh <= 1:
        return ""
    return f"_shard0of{nsh}" + ("" if slots is None else "_slots" + "-".join(map(str, slots)))


def load_pmc_traffic(cfg_name, nsh=1, slots=None, frame_out="rgb", kernel=None):
    """HBM bytes per launch of the dominant kernel from a PMC summary of the SAME
    configuration, rank share and kernel (profiles/pmc_<config><shard tag>.json,
    written from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes); None when
    there is none."""
    tag = cfg_name + shard_tag(nsh, slots) + ("" if frame_out == "rgb" else "_" + frame_out)
    p = os.path.join(ROOT, "profiles", f"pmc_{tag}.json")
    if os.path.exists(p):
        d = json.load(open(p))
        if d.get("config") == tag and (kernel is None or d.get("kernel", "").startswith(kernel)):
            return d.get("hbm_bytes_per_launch"), os.path.relpath(p, ROOT)
    return None, None


VERIFY_KEYS = ("verified", "warm_failures", "verify_digest", "verified_bands", "verified_buffers",
               "verify_mismatches", "verify_note", "fragments_match_oracle")
DIGEST_FILE = os.path.join(ROOT, "tests", "golden", "bench_digests.json")
BAND_ROWS = 32   # digest unit: one tile row (the tile-row shards' unit)


def band_digest(kind, a, W, H, b):
    """sha256[:32] of band b (rows [32b, 32b+32)) of one frame buffer: f64 / depth /
    u8 RGB rows, or for "yuv420p" the band's Y rows, then its U rows, then its V
    rows of the flat planes (tests/golden/make_bench_digests.py writes the oracle's)."""
    import hashlib
    r0, r1 = b * BAND_ROWS, min(H, (b + 1) * BAND_ROWS)
    if kind == "yuv420p":
        cw, ch = W // 2, H // 2
        a = np.asarray(a).reshape(-1)
        y = a[:W * H].reshape(H, W)
        u = a[W * H:W * H + cw * ch].reshape(ch, cw)
        v = a[W * H + cw * ch:W * H + 2 * cw * ch].reshape(ch, cw)
        data = y[r0:r1].tobytes() + u[r0 // 2:r1 // 2].tobytes() + v[r0 // 2:r1 // 2].tobytes()
    else:
        data = np.ascontiguousarray(a[r0:r1]).tobytes()
    return hashlib.sha256(data).hexdigest()[:32]


def anim_tx(i):
    """c3_animated's translate of frame i: a new sub-pixel offset every frame
    (a cycle of 100, never 0)."""
    return 0.005 + 0.01 * (i % 100)


# frame indices of c3_animated with committed oracle digests: the last timed
# frame of the driver's (--steps 20) and the default (100) run, and of the
# 11- and 12-frame loops of tests/test_bench_frames_gpu.py
ANIM_DIGEST_FRAMES = (10, 11, 19, 99)


def digest_key(cfg_name, cfg, frame_index):
    """Entry of bench_digests.json for the frame with this index (c3_animated:
    its transform depends on the frame index)."""
    return cfg_name + (f"@{frame_index % 100}" if cfg.get("animate") else "")


def load_digests():
    try:
        with open(DIGEST_FILE) as f:
            return json.load(f)
    except OSError:
        return {}


def host_cpu():
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model


def cpu_baseline(cfg, xy, z, c, budget_s=10.0, max_frames=50):
    """The oracle (CPU restatement, single thread) on the same frames, pinned
    to one core (sched_setaffinity, the equivalent of `taskset -c <cpu>`)."""
    import scenes
    f = scenes.OracleFactory()
    times, frags = [], 0
    ctx = f.context(cfg["W"], cfg["H"], False)
    old = os.sched_getaffinity(0)
    cpu = min(old)
    os.sched_setaffinity(0, {cpu})
    try:
        t_start = time.perf_counter()
        while len(times) < max_frames and (time.perf_counter() - t_start < budget_s or len(times) < 2):
            t0 = time.perf_counter()
            ctx.set_color(0, 0, 0, 0)
            ctx.set_depth_state(True, cfg.get("write", True))
            ctx.clear_depth()
            ctx.draw_triangles(xy, c, z=z)
            times.append(time.perf_counter() - t0)
            frags = ctx.last_fragment_count()
    finally:
        os.sched_setaffinity(0, old)
    med = float(np.median(times))
    return {"value": frags / med / 1e6, "unit": "Mpixels/s", "cores": 1, "kind": "port",
            "pinned_cpu": cpu, "host_cpu": host_cpu(), "host_nproc": os.cpu_count(),
            "host_affinity_cpus": len(old),
            "sample": f"{len(times)} full frames of the same workload, median {med*1e3:.1f} ms/frame "
                      f"(oracle/oracle.c, gcc -O3 -ffp-contract=off, 1 thread pinned to cpu {cpu} "
                      f"= taskset -c {cpu})"}


class Runner:
    """One configuration in one context: fragment count, breakdown pass, timed
    region (K frames, barrier + synchronize on both sides, max over ranks)."""

    def __init__(self, R, args, cfg_name, world, rank, dist, rdev, nsh, me, deliver="none", frame_output=None):
        self.R, self.args, self.cfg_name = R, args, cfg_name
        self.frame_output = frame_output or args.frame_output
        self.cfg = CONFIGS[cfg_name]
        self.world, self.rank, self.dist, self.rdev = world, rank, dist, rdev
        self.nsh, self.me, self.deliver = nsh, me, deliver
        cfg = self.cfg
        self.W, self.H = cfg["W"], cfg["H"]
        self.xy, self.z, self.c = make_scene(cfg)
        self.n_tri = len(self.xy)
        self.ctx = R.RenderContext(self.W, self.H, False)
        self.ctx.set_frame_format(self.frame_output)
        if args.force_ordered:
            self.ctx.set_force_ordered_raster(True)
        self.buf = R.TriangleBuffer(self.xy, self.c, z=self.z, gouraud=cfg["gouraud"])
        self.comm = None
        self.host = None
        self.tickets = []
        if deliver == "host":
            nbytes = int(np.prod(self.ctx.frame_output_shape()))
            self.host = [R.HostBuffer(nbytes) for _ in range(2)]
        elif deliver == "bands":
            # every rank copies its own bands into one host frame (two, in
            # turn): shared pinned memory across the ranks' processes at N > 1
            nbytes = int(np.prod(self.ctx.frame_output_shape()))
            if world > 1:
                tag = os.environ.get("MASTER_PORT", "0")
                names = [f"/nr_bench_frame{j}_{tag}" for j in range(2)]
                if rank == 0:
                    self.host = [R.SharedHostBuffer(nm, nbytes, owner=True) for nm in names]
                dist.barrier()
                if rank != 0:
                    self.host = [R.SharedHostBuffer(nm, nbytes) for nm in names]
                dist.barrier()
            else:
                self.host = [R.HostBuffer(nbytes) for _ in range(2)]
        self.fixed_k = None if args.root_slots in ("auto", "equal") else int(args.root_slots)
        self.root_k = self.fixed_k
        self.apply_partition(self.fixed_k)

    def slots_for(self, k):
        return None if k is None else [k] + [2] * (self.nsh - 1)

    def apply_partition(self, k):
        if self.nsh <= 1:
            return
        if k is None:
            self.ctx.set_shard(self.nsh, self.me)
        else:
            self.ctx.set_shard_slots(self.nsh, self.me, self.slots_for(k))

    def frame(self, i=0):
        ctx = self.ctx
        ctx.set_color(0, 0, 0, 0)
        ctx.set_depth_state(True, self.cfg.get("write", True))
        ctx.clear_depth()
        if self.cfg.get("animate"):   # a new transform every frame: the binning key changes
            ctx.save_state()
            ctx.translate(anim_tx(i), 0.0)
            ctx.draw_triangle_buffer(self.buf)
            ctx.restore_state()
        else:
            ctx.draw_triangle_buffer(self.buf)
        if self.deliver == "bands":
            # no gather: this rank's bands straight into the host frame; host
            # frame i % 2 is rewritten only after frame i-2's copies landed
            if len(self.tickets) >= 2:
                ctx.wait_frame_delivered(self.tickets.pop(0))
            self.tickets.append(ctx.deliver_frame_bands(self.host[i % 2]))
            return
        ctx.gather_frame_u8(self.comm, 0)
        if self.host is not None and self.rank == 0:
            # frame i's D2H runs on the gather stream while frame i+1 renders;
            # host buffer i % 2 is rewritten only after frame i-2 has landed
            if len(self.tickets) >= 2:
                ctx.wait_frame_delivered(self.tickets.pop(0))
            self.tickets.append(ctx.deliver_frame(self.host[i % 2]))

    def drain(self):
        self.ctx.flush()
        while self.tickets:
            self.ctx.wait_frame_delivered(self.tickets.pop(0))

    def sync(self):
        import torch
        torch.cuda.synchronize()
        if self.dist is not None:
            self.dist.barrier()

    def max_over_ranks(self, v):
        if self.dist is None:
            return v
        import torch
        t = torch.tensor([v], device=self.rdev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def verify(self, last_i):
        """After the timed region: the last timed frame read back and checked,
        band by band, against the oracle's digests of the same frame
        (tests/golden/bench_digests.json) -- the f64 framebuffer and u32 depth
        of this rank's owned bands, the frame output on the device (every band
        on the gathering root, the owned ones elsewhere) and, when the frame is
        delivered to host memory, the host frame of the last step.  Also the
        warm binning's failure count (a failed warm batch falls back to an exact
        but slower raster), which must be 0."""
        from libnativecpurenderer_amd import sharding
        ctx = self.ctx
        out = {"verified": None, "warm_failures": int(ctx.warm_failure_count())}
        key = digest_key(self.cfg_name, self.cfg, last_i)
        ref = load_digests().get(key)
        if ref is None or (ref["W"], ref["H"], ref["band_rows"]) != (self.W, self.H, BAND_ROWS):
            out["verify_note"] = f"no oracle digest for {key}"
            return out
        nb = (self.H + BAND_ROWS - 1) // BAND_ROWS
        slots = self.slots_for(self.root_k) if self.nsh > 1 else None
        owned = ([y0 // BAND_ROWS for y0, _ in sharding.owned_bands(self.H, self.nsh, self.me, slots=slots)]
                 if self.nsh > 1 else list(range(nb)))
        fo = self.frame_output
        # the frame output on the device: the whole frame on the root of an RCCL
        # gather; the host frame: whole too when every rank delivered its bands
        # into it (drain + barrier before this runs)
        dev_bands = list(range(nb)) if (self.world > 1 and self.comm is not None and self.rank == 0) else owned
        host_bands = list(range(nb)) if (self.deliver == "bands" and self.world > 1) else dev_bands
        checks = [("f64", "f64", ctx.get_buffer_numpy(), owned), ("depth", "depth", ctx.get_depth_buffer(), owned)]
        if self.deliver != "bands":
            checks.append(("frame_output", fo, ctx.get_frame_u8(), dev_bands))
        if self.host is not None and self.rank == 0:   # the host frame of the last step
            hb = np.asarray(self.host[last_i % 2].array()).reshape(-1)[:int(np.prod(ctx.frame_output_shape()))]
            a = hb if fo == "yuv420p" else hb.reshape(ctx.frame_output_shape())
            checks.append(("host_frame", fo, a, host_bands))
        bad, n = [], 0
        for what, kind, arr, bands in checks:
            for b in bands:
                n += 1
                if band_digest(kind, arr, self.W, self.H, b) != ref[kind][b]:
                    bad.append(f"{what}:band{b}")
        out.update({"verified": not bad, "verify_digest": f"{os.path.relpath(DIGEST_FILE, ROOT)}[{key}]",
                    "verified_bands": n, "verified_buffers": [c[0] for c in checks]})
        if bad:
            out["verify_mismatches"] = bad[:16]
        if self.nsh == 1 and self.world == 1 and not self.cfg.get("animate"):
            out["fragments_match_oracle"] = int(round(self.frags)) == ref["fragments"]
        return out

    def run(self, steps, warmup, calibrate=False):
        import torch
        ctx, dist = self.ctx, self.dist
        # fragment count of one frame (outside the timed region), summed over
        # ranks; an animated workload: the mean over two of its transforms
        ctx.set_fragment_counting(True)
        nf = 2 if self.cfg.get("animate") else 1
        for i in range(nf):
            self.frame(i)
        self.drain()
        frags = ctx.get_fragment_count() / nf
        ctx.set_fragment_counting(False)
        if dist is not None:
            t = torch.tensor([frags], dtype=torch.float64, device=self.rdev)
            dist.all_reduce(t)
            frags = float(t.item())
        self.frags = frags

        # partition calibration (N>1, --root-slots auto): every candidate share
        # of rank 0 is timed over a few frames (max over ranks), the fastest kept
        calib = {}
        if calibrate:
            for k in (None, 3, 4, 5, 6, 8, 10, 12):
                self.apply_partition(k)
                for _ in range(3):
                    self.frame()
                self.drain()
                self.sync()
                t0 = time.perf_counter()
                for i in range(10):
                    self.frame(i)
                self.drain()
                torch.cuda.synchronize()
                calib["equal" if k is None else str(k)] = round(self.max_over_ranks(time.perf_counter() - t0) / 10 * 1e3, 4)
            best = min(calib, key=calib.get)
            self.root_k = None if best == "equal" else int(best)
            self.apply_partition(self.root_k)

        # clock settle (CLOCK_SETTLE_MS of frames, untimed), then the W warmup steps
        self.sync()
        t0, nset = time.perf_counter(), 0
        while self.max_over_ranks((time.perf_counter() - t0) * 1e3) < self.args.clock_settle_ms:
            for i in range(4):   # (every rank the same frames: N > 1 frames end in a collective)
                self.frame(i)
            nset += 4
            self.drain()
        self.settle_frames = nset
        for i in range(warmup):
            self.frame(i)
        self.drain()

        names = ("tri_count", "tri_scan", "tri_emit", "tri_sort", "tile_ranges", "vis_init", "tile_raster",
                 "resolve", "fill", "output", "gather")
        # (1) breakdown pass: HIP events around every kernel (they add launch
        #     gaps, so this pass is not the headline)
        ctx.reset_kernel_timing()
        ctx.set_kernel_timing_filter("")
        ctx.enable_kernel_timing(True)
        for i in range(steps):
            self.frame(i)
        self.drain()
        ctx.enable_kernel_timing(False)
        kernels = {}
        for name in names:
            tot, cnt = ctx.get_kernel_timing(name)
            if cnt:
                kernels[name] = round(tot / cnt * 1e3, 2)   # us per launch
        path = ctx.last_raster_path()
        from libnativecpurenderer_amd import sharding
        slots = self.slots_for(self.root_k) if self.nsh > 1 else None
        share = len(sharding.owned_rows(self.H, self.nsh, self.me, slots=slots)) / self.H
        kb = kernel_bytes(self.cfg, self.n_tri, path, share, self.frame_output)
        dom = max((k for k in kb if k in kernels), key=lambda k: kernels[k])

        # (2) kernel pass: K frames with only the dominant kernel timed: the
        #     raster stamps its own execution span on the device's 100 MHz
        #     clock (first workgroups' start, last workgroup's end; no packet
        #     on the stream -- events around or bound to the launch also
        #     counted the launch gap, profiles/r06/ab_event_every.txt).  The
        #     timed region below carries no timing at all.
        dom_us, cnt = kernels[dom], 0
        if not self.args.no_kernel_timing:
            ctx.reset_kernel_timing()
            ctx.set_kernel_timing_filter(dom)
            ctx.enable_kernel_timing(True)
            for i in range(steps):
                self.frame(i)
            self.drain()
            ctx.enable_kernel_timing(False)
            tot, cnt = ctx.get_kernel_timing(dom)
            if cnt:
                dom_us = round(tot / cnt * 1e3, 2)
            ctx.reset_kernel_timing()

        # (3) timed region: K frames, nothing but the frames
        self.sync()
        warm0, loose0 = ctx.warm_batch_count(), ctx.loose_batch_count()
        t0 = time.perf_counter()
        for i in range(steps):
            self.frame(i)
        self.drain()
        torch.cuda.synchronize()
        dt = self.max_over_ranks(time.perf_counter() - t0)
        if dist is not None:
            dist.barrier()
        warm_frames = ctx.warm_batch_count() - warm0
        loose_frames = ctx.loose_batch_count() - loose0
        ms = dt / steps * 1e3
        # the last timed frame against the oracle's digests (outside the timed region)
        ver = self.verify(steps - 1)
        if dist is not None:   # every rank's verdict: false if any rank mismatched
            if self.max_over_ranks(1.0 if ver["verified"] is False else 0.0) > 0:
                ver["verified"] = False
            ver["warm_failures"] = int(self.max_over_ranks(float(ver["warm_failures"])))
        achieved = kb[dom] / (dom_us * 1e-6) / 1e9
        B = algorithmic_bytes(self.cfg, self.n_tri, frame_out=self.frame_output)   # whole frame
        ksym = "k_tile_raster" if path == "ordered" else "k_vis"
        # (at N>1 the PMC summary of rank 0's share, taken as an emulated share on one GPU)
        traffic, traffic_src = load_pmc_traffic(self.cfg_name, self.nsh, slots, self.frame_output, ksym)
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": PEAK_HBM_GBPS, "unit": "GB/s",
                "frac": round(achieved / PEAK_HBM_GBPS, 4), "traffic": traffic,
                "traffic_source": traffic_src or "none for this config/share (null)",
                # the bytes the kernel physically moved (PMC) over the same kernel time
                "traffic_frac": round(traffic / (dom_us * 1e-6) / 1e9 / PEAK_HBM_GBPS, 4) if traffic else None,
                "kernel": KERNEL_SYMBOL[dom], "kernel_us": dom_us,
                "kernel_us_source": (f"device-clock span (s_memrealtime) of {cnt} launches, a K-frame pass before "
                                     f"the timed region" if cnt else "breakdown pass"),
                "algorithmic_bytes_per_launch": kb[dom], "rank_share_of_frame": round(share, 6),
                **frame_roofline(B, share, ms, self.world)}
        out = {
            "value": round(frags * steps / dt / 1e6, 1),
            "ms_per_step": round(ms, 4),
            "fps": round(1e3 / ms, 1),
            "fragments_per_frame": int(round(frags)),
            "roofline": roof,
            "raster_path": path,
            "kernel_us": kernels,
            "slots": slots,
            "calib": calib,
            "warm_binned_frames": warm_frames,
            "loose_binned_frames": loose_frames,
            "clock_settle": {"ms": self.args.clock_settle_ms, "frames": self.settle_frames},
            **ver,
        }
        if path == "ordered" and self.cfg.get("soup", (0, 0, None))[2] is not None:
            # C5: the blend loop is bound by f64 VALU issue, not by HBM (per
            # rank: frags is this context's count at N=1, the ranks' sum at N>1)
            ops = (frags if self.world == 1 else frags / self.world) * BLEND_OPS_PER_FRAGMENT
            tops = ops / (dom_us * 1e-6) / 1e12
            out["valu_roofline"] = {"bound": "valu", "achieved": round(tops, 3), "peak": round(PEAK_F64_VALU_TOPS, 2),
                                    "unit": "Top/s (f64 add/mul lanes)", "frac": round(tops / PEAK_F64_VALU_TOPS, 4),
                                    "ops_per_fragment": BLEND_OPS_PER_FRAGMENT,
                                    "note": "blended fragments x 6 f64 ops / k_tile_raster time; peak = 256 CU x 4 SIMD "
                                            "x 16 f64 lanes/clk x 2.4 GHz"}
        return out


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20,
                    help="untimed warmup steps (after the clock settle, --clock-settle-ms)")
    ap.add_argument("--clock-settle-ms", type=float, default=CLOCK_SETTLE_MS,
                    help="untimed frames first, until the GPU has rendered this long (its clocks ramp after idle), "
                         "then the --warmup steps")
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--extra", dest="extra", action="store_true", default=None,
                    help="also time the metric's literal config (1M tris at 1080p), c2, c5 and host-delivered "
                         "frames, reported under 'extra' (default at N=1)")
    ap.add_argument("--no-extra", dest="extra", action="store_false")
    ap.add_argument("--deliver", default="none", choices=("none", "host", "bands"),
                    help="host: every step ends with the frame output on the host (pinned buffers, D2H of frame k "
                         "overlapped with frame k+1), as the video caller (PutRendererContextFrame) needs it; "
                         "bands: every rank copies its own bands straight into one shared pinned host frame "
                         "(DeliverFrameBands, no GPU gather: each GPU's PCIe link carries its share)")
    ap.add_argument("--no-kernel-timing", action="store_true", help="time without per-kernel HIP events")
    ap.add_argument("--force-ordered", action="store_true", help="A/B: always take the in-order tile raster")
    ap.add_argument("--lib", default=None,
                    help="experiment: load another build of the library (tools/exp A/B and probe builds)")
    ap.add_argument("--emulate-shards", type=int, default=0,
                    help="experiment: render shard 0 of N on this one GPU (no gather) to time one rank's share")
    ap.add_argument("--gloo-test", action="store_true",
                    help="testing the N>1 orchestration on one GPU: gloo process group, CPU reductions, every rank "
                         "renders its shard on its LOCAL_RANK device but the RCCL frame gather is skipped")
    ap.add_argument("--frame-output", default="yuv420p", choices=sorted(FRAME_OUT_BPP),
                    help="frame output of every step: the YUV420P planes (default since round 5: the video encoder's "
                         "input, PutRendererContextFrame cpp:232-275 -- 1.5 B/px, which halves the root's ingress "
                         "at N>1) or the u8 image (cpp:52-57, 3 B/px; the headline's output in rounds 1-4), written "
                         "by the raster and gathered")
    ap.add_argument("--root-slots", default="auto",
                    help="N>1 (and --emulate-shards): tile-row share of rank 0, in bands per 2 bands of every other "
                         "rank (SetShardSlots); 'equal' = SetShard; 'auto' (N>1) times candidates and keeps the "
                         "fastest -- the root also receives every other rank's bands, so it gets less to render "
                         "when the gather dominates")
    return ap.parse_args(argv)


def main():
    args = parse_args()
    if args.lib:
        from libnativecpurenderer_amd import _lib
        _lib.LIB_PATH = os.path.abspath(args.lib)

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

    nsh = world if world > 1 else max(1, args.emulate_shards)
    me = rank if world > 1 else 0
    run = Runner(R, args, args.config, world, rank, dist, rdev, nsh, me, args.deliver)
    if world > 1 and not args.gloo_test:
        from libnativecpurenderer_amd import sharding
        run.comm = sharding.make_comm(dist, world, rank)
    res = run.run(args.steps, args.warmup, calibrate=world > 1 and args.root_slots == "auto")

    extra = {}
    do_extra = args.extra if args.extra is not None else (world == 1 and nsh == 1)
    if do_extra and world == 1:
        jobs = [("c3_1080p", "none", None), ("c3_animated", "none", None), ("c2", "none", None), ("c5", "none", None),
                (args.config, "none", "rgb"), (args.config, "host", None), (args.config, "host", "rgb"),
                ("c2", "host", None)]
        for name, dl, fo in jobs:
            if name == args.config and dl == args.deliver and (fo or args.frame_output) == args.frame_output:
                continue
            sub = Runner(R, args, name, 1, 0, None, rdev, nsh, 0, dl, fo)
            r = sub.run(args.steps, args.warmup)
            key = name + ("_host_delivered" if dl == "host" else "") + ("_" + fo if fo else "")
            what = (" + frame output (" + ("YUV420P planes, the encoder's input" if sub.frame_output == "yuv420p"
                                           else "u8 RGB image") + ") delivered to host memory") if dl == "host" else ""
            extra[key] = {"workload": sub.cfg["desc"] + what,
                          "triangles": sub.n_tri, **{k: r[k] for k in ("value", "ms_per_step", "fps",
                                                                         "fragments_per_frame", "roofline",
                                                                         "raster_path", "kernel_us",
                                                                         "warm_binned_frames",
                                                                         "loose_binned_frames")},
                          **{k: r[k] for k in VERIFY_KEYS if k in r},
                          **({"valu_roofline": r["valu_roofline"]} if "valu_roofline" in r else {})}
            if name == "c3_1080p" and dl == "none" and not args.no_cpu_baseline:
                # the metric's literal configuration gets its own CPU baseline (same oracle, same pinning)
                extra[key]["cpu_baseline"] = cpu_baseline(sub.cfg, sub.xy, sub.z, sub.c, budget_s=5.0)
                extra[key]["vs_cpu"] = round(r["value"] / extra[key]["cpu_baseline"]["value"], 1)
            if dl == "host":
                extra[key]["host_frame_bytes"] = int(np.prod(sub.ctx.frame_output_shape()))
                same = res if name == args.config and args.deliver == "none" else extra.get(name)
                extra[key]["in_hbm_ms_per_step"] = same["ms_per_step"] if same else None
            del sub
        # the real caller's frame: milrenderer's primitive mix (milrenderer.py:865-1038) through the deferred
        # command list, with its frame handed over as YUV420P in host memory, beside the oracle
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import bench_mil
        extra["milrenderer_command_list"] = bench_mil.run(frames=max(10, min(args.steps, 50)),
                                                          oracle=not args.no_cpu_baseline)

    if rank != 0:
        return
    cfg = run.cfg
    result = {
        "metric": "Mpixels/s shaded+Z-tested (and fps)",
        "value": res["value"],
        "unit": "Mpixels/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": res["ms_per_step"],
        "fps": res["fps"],
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (deterministic displaced UV sphere / seeded soup, SURVEY.md §8d)",
        "config": {"workload": cfg["desc"], "width": run.W, "height": run.H, "triangles": run.n_tri,
                   "fragments_per_frame": res["fragments_per_frame"], "frame_pixels": run.W * run.H,
                   "frame_output": args.frame_output,
                   "frame_delivery": {"host": "host (pinned, D2H overlapped)",
                                      "bands": "host, each rank's own bands into one shared pinned host frame "
                                               "(DeliverFrameBands, no gather)"}.get(args.deliver, "in HBM"),
                   "parallelism": (f"tile-row shards x{world} + " + ("bands into a shared host frame" if args.deliver == "bands" else "RCCL u8 frame gather") if world > 1
                                   else f"EMULATED shard 0 of {nsh} on one GPU (no gather)" if nsh > 1
                                   else "single GPU"),
                   **({"shard_slots": res["slots"] or "equal", "partition_calibration_ms": res["calib"]}
                      if nsh > 1 else {})},
        "roofline": res["roofline"],
        "raster_path": res["raster_path"],
        "kernel_us": res["kernel_us"],
        "clock_settle": res["clock_settle"],
        **{k: res[k] for k in VERIFY_KEYS if k in res},
        "kernel_us_note": "kernel_us: per-launch averages from a breakdown pass with events around every kernel "
                          "(the rasters by their device-clock span); roofline.kernel_us: the dominant kernel's "
                          "device-clock span over a K-frame pass of its own (roofline.kernel_us_source); the "
                          "timed region carries no timing",
    }
    if "valu_roofline" in res:
        result["valu_roofline"] = res["valu_roofline"]
    if extra:
        result["extra"] = extra
    if not args.no_cpu_baseline and world == 1:
        result["cpu_baseline"] = cpu_baseline(cfg, run.xy, run.z, run.c)
        result["vs_cpu"] = round(result["value"] / result["cpu_baseline"]["value"], 1)
    print(json.dumps(result))


if __name__ == "__main__":
    main()
