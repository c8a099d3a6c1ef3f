"""Oracle digests of the frames bench.py times (tests/golden/bench_digests.json).

bench.py verifies the last frame of its timed region against these digests
after the timed region (Runner.verify): the f64 framebuffer, the u32 depth
buffer and the frame output (u8 RGB image, cpp:52-57, and its YUV420P planes)
of every configuration in bench.CONFIGS, rendered here by the CPU oracle
(oracle/oracle.c: clear, depth clear, DrawTriangles -- the frame loop of
src/milrenderer.py:865-1038 reduced to the triangle path).  The GPU box has no
oracle run inside bench.py's product leg, so the oracle's result travels as
digests.

Per 32-row band (a tile row, the unit of the tile-row shards):
sha256[:32] of the band's f64 rows, depth rows, u8 RGB rows and YUV420P rows
(Y rows of the band, then its U rows, then its V rows).  Any rank share is
checked as the digests of the bands it owns; a whole frame as all of them.

c3_animated translates by bench.anim_tx(i) in frame i: one entry per frame
index in bench.ANIM_DIGEST_FRAMES.

    python tests/golden/make_bench_digests.py [config ...]
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
OUT = os.path.join(HERE, "bench_digests.json")
BAND = 32   # rows per tile row (nr_common.h TH)


def _bench():
    spec = importlib.util.spec_from_file_location("bench_for_digests", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def band_digests(b, f64, depth, u8, yuv, W, H):
    """Per-band digests of one frame's buffers (bench.band_digest: the layout
    bench.Runner.verify reads back)."""
    nb = (H + BAND - 1) // BAND
    return {kind: [b.band_digest(kind, a, W, H, k) for k in range(nb)]
            for kind, a in (("f64", f64), ("depth", depth), ("rgb", u8), ("yuv420p", yuv))}


def oracle_frame(cfg, xy, z, c, tx=0.0):
    """One bench frame on the oracle (bench.Runner.frame's calls; tx: the
    animated workload's translate)."""
    import scenes
    ctx = scenes.OracleFactory().context(cfg["W"], cfg["H"], False)
    ctx.set_color(0, 0, 0, 0)
    ctx.set_depth_state(True, cfg.get("write", True))
    ctx.clear_depth()
    if cfg.get("animate"):
        ctx.save_state()
        ctx.translate(tx, 0.0)
        ctx.draw_triangles(xy, c, z=z)
        ctx.restore_state()
    else:
        ctx.draw_triangles(xy, c, z=z)
    u8 = ctx.get_buffer_as_uint8_numpy()
    return (ctx.get_buffer_numpy(), ctx.get_depth_buffer(), u8, scenes.yuv420p(u8), ctx.last_fragment_count())


def make(configs=None):
    b = _bench()
    data = json.load(open(OUT)) if os.path.exists(OUT) else {}
    data["_about"] = ("oracle digests of bench.py's frames, tests/golden/make_bench_digests.py: per 32-row band "
                      "sha256[:32] of the f64 framebuffer, u32 depth, u8 RGB and YUV420P rows")
    for name in configs or sorted(b.CONFIGS):
        cfg = b.CONFIGS[name]
        xy, z, c = b.make_scene(cfg)
        for fi in (b.ANIM_DIGEST_FRAMES if cfg.get("animate") else (0,)):
            t0 = time.time()
            f64, depth, u8, yuv, frags = oracle_frame(cfg, xy, z, c, b.anim_tx(fi) if cfg.get("animate") else 0.0)
            assert b.BAND_ROWS == BAND
            d = band_digests(b, f64, depth, u8, yuv, cfg["W"], cfg["H"])
            key = b.digest_key(name, cfg, fi)
            data[key] = {"W": cfg["W"], "H": cfg["H"], "band_rows": BAND, "triangles": int(len(xy)),
                         "fragments": int(frags), **d}
            print(f"{key}: {frags} fragments, {time.time() - t0:.1f} s", flush=True)
    with open(OUT, "w") as f:
        json.dump(data, f, indent=0, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    make(sys.argv[1:] or None)
