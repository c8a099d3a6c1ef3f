"""milrenderer-style frame benchmark: the per-frame primitive
mix of milrenderer.py:865-1038 (background texture, dim fill, gradient bands,
judge lines with heads, tap/hold notes under per-note transforms, hit
effects) at 1920x1080 RGB, synthetic textures and positions.  Times one
frame drawn (a) with immediate calls (one launch per draw), (b) recorded as a
deferred command list (one launch per frame), (c) by the CPU oracle (1
thread); checks (b) against (c) bit for bit.  Prints one JSON line."""
import argparse, json, math, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np
import scenes

W, H = 1920, 1080


def make_textures(fac):
    return dict(bg=fac.texture(scenes.pattern_u8(H, W, 3, seed=1)),
                head=fac.texture(scenes.pattern_u8(64, 64, 4, seed=2)),
                note=fac.texture(scenes.pattern_u8(32, 128, 4, seed=3)),
                hold=fac.texture(scenes.pattern_u8(32, 96, 4, seed=4)),
                hit=fac.texture(scenes.pattern_u8(256, 256, 4, seed=5)))


def plan(t, nlines=8, nnotes=300, nhits=40):
    """The frame's varying numbers (note positions, rotations, hold lengths,
    hit effects), drawn from a seeded generator before the timed region: the
    timed region then measures the draw calls, not numpy's per-call RNG
    overhead (~1 us per uniform() call, ~900 per frame)."""
    r = np.random.Generator(np.random.PCG64(1000 + int(t * 100)))
    lines = []
    for k in range(nlines):
        cx, cy = float(r.uniform(0.2 * W, 0.8 * W)), float(r.uniform(0.3 * H, 0.7 * H))
        rot = float(r.uniform(-30, 30)) + 20 * math.sin(t + k)
        notes = []
        for n in range(nnotes // nlines):
            tx_, ty_ = float(r.uniform(-400, 400)), float(r.uniform(-600, 0))
            notes.append((tx_, ty_, None if n % 5 else float(r.uniform(60, 300))))
        lines.append((cx, cy, rot, math.cos(math.radians(rot)) * W, math.sin(math.radians(rot)) * W, notes))
    hits = [(float(r.uniform(0, W)), float(r.uniform(0, H)), float(r.uniform(0, 360)), float(r.uniform(0.3, 1)))
            for _ in range(nhits)]
    return lines, hits


def frame(ctx, tx, fp):
    """milrenderer.py:865-1038's per-frame call sequence over plan() `fp`."""
    lines, hits = fp
    ctx.set_color(0, 0, 0, 0)
    ctx.draw_texture(tx["bg"], 0, 0, W, H)
    ctx.fill_color(0, 0, 0, 0.6)
    ctx.draw_vertical_mut_grd(0, H * 0.6, W, H * 0.4, [(0.0, (0, 0, 0, 0)), (0.3, (0.1, 0.1, 0.2, 0.3)),
                                                     (0.7, (0.1, 0.1, 0.3, 0.5)), (1.0, (0, 0, 0, 0.7))])
    head, note, hold = tx["head"], tx["note"], tx["hold"]
    for cx, cy, rot, dx, dy, notes in lines:
        ctx.save_state()
        ctx.draw_texture(head, cx - 24, cy - 24, 48, 48)
        ctx.restore_state()
        ctx.draw_line(cx - dx, cy - dy, cx + dx, cy + dy, 4.0, 1, 1, 1, 0.8)
        ctx.save_state()
        ctx.translate(cx, cy)
        ctx.rotate_degree(rot - 90)
        for ntx, nty, L in notes:
            ctx.save_state()
            ctx.translate(ntx, nty)
            ctx.rotate_degree(90)
            ctx.scale(1.2, 1.2)
            if L is None:
                ctx.draw_texture(note, -16, -64, 32, 128)
            else:
                ctx.draw_splitted_texture(hold, -20, -64, 21, 128, 0, 0.2, 0, 1)
                ctx.draw_splitted_texture(hold, 0, -64, L + 1, 128, 0.2, 0.8, 0, 1)
                ctx.draw_splitted_texture(hold, L, -64, 21, 128, 0.8, 1.0, 0, 1)
            ctx.restore_state()
        ctx.restore_state()
    hit = tx["hit"]
    for hx, hy, hr, ha in hits:
        ctx.save_state()
        ctx.translate(hx, hy)
        ctx.rotate_degree(hr)
        ctx.apply_color_transform(1, 1, 1, ha)
        ctx.draw_texture(hit, -90, -90, 180, 180)
        ctx.restore_state()


class Counter:
    """Counts the draw calls of a frame (no drawing)."""
    def __init__(self): self.n = 0; self.calls = 0
    def __getattr__(self, name):
        def f(*a):
            if name.startswith("draw") or name in ("fill_color", "set_color"): self.n += 1
            self.calls += 1
        return f
    def draw_vertical_mut_grd(self, x, y, w, h, steps): self.n += len(steps) - 1; self.calls += len(steps) - 1


def run(frames=30, oracle=True):
    """One JSON-able dict: ms per frame for immediate calls, the recorded
    command list (one call per draw / state op), the recorded list with the
    whole frame packed into one ExecuteCommands call (PackedCommands), the
    packed frame handed to the video caller (YUV420P planes,
    PutRendererContextFrame's input, cpp:232-275, delivered to host memory,
    D2H overlapped with the next frame), and the CPU oracle; the recorded and
    packed frames checked against the oracle bit for bit."""
    from libnativecpurenderer_amd import libNativeCPURendererPybind as R
    gpu = scenes.GpuFactory()
    tx = make_textures(gpu)
    plans = [plan(i * 0.1) for i in range(max(frames, 3))]
    last = plan(0.7)
    cnt = Counter()
    frame(cnt, {k: None for k in tx}, plans[0])
    res = {"workload": "milrenderer-style frame 1920x1080 RGB (milrenderer.py:865-1038 primitive mix)",
           "draws_per_frame": cnt.n, "calls_per_frame": cnt.calls,
           "note": "frame parameters drawn before the timed region (plan()); the timed region is the API calls"}
    outs = {}
    for mode in ("immediate", "recorded", "packed", "packed_yuv420p_to_host"):
        ctx = R.RenderContext(W, H, False)
        host, tickets = None, []
        if mode != "immediate":
            ctx.begin_commands()
        front = ctx.packed() if mode.startswith("packed") else ctx
        if mode == "packed_yuv420p_to_host":
            ctx.set_frame_format("yuv420p")
            host = [R.HostBuffer(int(np.prod(ctx.frame_output_shape()))) for _ in range(2)]

        def one(i, fp):
            frame(front, tx, fp)
            if front is not ctx:
                front.submit()
            if mode != "immediate":
                ctx.flush_commands()
            if host is not None:
                ctx.gather_frame_u8()
                if len(tickets) >= 2:
                    ctx.wait_frame_delivered(tickets.pop(0))
                tickets.append(ctx.deliver_frame(host[i % 2]))

        for i in range(3):
            one(i, plans[i])
        ctx.flush()
        while tickets:
            ctx.wait_frame_delivered(tickets.pop(0))
        t0 = time.perf_counter()
        for i in range(frames):
            one(i, plans[i])
        ctx.flush()
        while tickets:
            ctx.wait_frame_delivered(tickets.pop(0))
        dt = (time.perf_counter() - t0) / frames
        res[f"{mode}_ms_per_frame"] = round(dt * 1e3, 3)
        if mode in ("recorded", "packed"):
            ctx.enable_kernel_timing(True)
            one(0, plans[1])
            ctx.flush()
            tot, c = ctx.get_kernel_timing("prim")
            res[f"{mode}_launch_us"] = round(tot / max(c, 1) * 1e3, 1)
            ctx.enable_kernel_timing(False)
            one(0, last)
            outs[mode] = ctx.get_buffer_numpy()
    if oracle:
        of = scenes.OracleFactory()
        otx = make_textures(of)
        octx = of.context(W, H, False)
        t0 = time.perf_counter()
        frame(octx, otx, last)
        o = octx.get_buffer_numpy()
        res["oracle_ms_per_frame"] = round((time.perf_counter() - t0) * 1e3, 1)
        res["oracle_note"] = "CPU oracle (oracle/oracle.c, 1 thread), the same frame's draws; no frame output"
        for mode, g in outs.items():
            res[f"{mode}_bit_exact_vs_oracle"] = bool(scenes.bits_equal(g, o))
        res["verified"] = all(res[f"{mode}_bit_exact_vs_oracle"] for mode in outs)
    else:
        res["verified"] = None
        res["verify_note"] = "the oracle check runs with the CPU baseline (--no-cpu-baseline skips both)"
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=30)
    ap.add_argument("--no-oracle", action="store_true")
    args = ap.parse_args()
    print(json.dumps(run(args.frames, not args.no_oracle)))


if __name__ == "__main__":
    main()
