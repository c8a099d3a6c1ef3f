"""CPU model of k_vis's raster-loop divergence on a scene (C3 by default).

Per (triangle, tile) pair: its rows in the tile and the span of each row
(ceil-crossing rule).  Tile lists in triangle order, 64-pair
chunks.  Reports, per model, the wave-iteration counts of the raster loop:

  nested : for k < max rows (lane-relative): one span step + max over lanes of
           ceil(span/2) pixel steps (today's loop)
  flat   : one loop whose iteration is "a span step if the lane's row is done,
           then one pixel pair": iterations = max over lanes of
           sum over its rows of max(1, ceil(span/2))
  ideal  : lane-parallel over fragments: pairs of fragments / 64 per chunk

Usage: python tools/exp/sim_chunks.py [W H rows cols]
"""
import math
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/tests")
import scenes  # noqa: E402

TW, TH = 64, 32


def main():
    W, H, rows, cols = (int(a) for a in sys.argv[1:5]) if len(sys.argv) > 4 else (3840, 2160, 500, 1000)
    xy, z, c = scenes.sphere_mesh(W, H, rows, cols)
    n = xy.shape[0]
    sx = xy[:, 0::2]
    sy = xy[:, 1::2]
    ymn, ymx = sy.min(1), sy.max(1)
    xmn, xmx = sx.min(1), sx.max(1)
    # pixel rows with a straddling edge: ceil(ymin) <= y < ceil(ymax)
    ya = np.clip(np.ceil(ymn), 0, H).astype(np.int64)
    yb = np.clip(np.ceil(ymx), 0, H).astype(np.int64)
    nrow = yb - ya
    tri = np.repeat(np.arange(n), nrow)
    y = (np.repeat(ya - np.cumsum(np.r_[0, nrow[:-1]]), nrow) + np.arange(nrow.sum())).astype(np.float64)
    # crossings of the 3 edges at y (half-open straddle rule)
    X0, Y0 = sx[tri], sy[tri]
    cr = np.full((len(tri), 3), np.nan)
    for k in range(3):
        i, j = k, (k + 1) % 3
        xi, yi, xj, yj = X0[:, i], Y0[:, i], X0[:, j], Y0[:, j]
        st = (yi > y) != (yj > y)
        with np.errstate(divide="ignore", invalid="ignore"):
            xc = (xj - xi) * (y - yi) / (yj - yi) + xi
        cr[st, k] = xc[st]
    lo = np.ceil(np.nanmin(cr, 1))
    hi = np.ceil(np.nanmax(cr, 1))
    lo = np.nan_to_num(lo, nan=0).astype(np.int64)
    hi = np.nan_to_num(hi, nan=0).astype(np.int64)
    lo = np.clip(lo, 0, W)
    hi = np.clip(hi, 0, W)
    yi = y.astype(np.int64)
    ty = yi // TH
    # split each row's span by tile columns
    tx0 = lo // TW
    tx1 = np.maximum((hi - 1) // TW, tx0)
    ncol = tx1 - tx0 + 1
    rr = np.repeat(np.arange(len(tri)), ncol)
    txs = np.repeat(tx0, ncol) + (np.arange(ncol.sum()) - np.repeat(np.cumsum(np.r_[0, ncol[:-1]]), ncol))
    seg_lo = np.maximum(lo[rr], txs * TW)
    seg_hi = np.minimum(hi[rr], (txs + 1) * TW)
    span = np.maximum(seg_hi - seg_lo, 0)
    seg_tri = tri[rr]
    seg_tile = ty[rr] * (W // TW + (W % TW > 0)) + txs
    seg_row = yi[rr] % TH
    print(f"triangles {n}  rows {len(tri)}  segments {len(rr)}  fragments {span.sum()}")
    # (triangle, tile) pairs: rows of the pair in the tile (the loop walks every straddled row of the tile's
    # row range, including rows whose span misses this tile column -> those are span steps with 0 pixels)
    key = seg_tile * n + seg_tri
    order = np.argsort(key, kind="stable")
    key_s = key[order]
    span_s = span[order]
    brk = np.r_[0, np.flatnonzero(np.diff(key_s)) + 1, len(key_s)]
    npair = len(brk) - 1
    pair_tile = key_s[brk[:-1]] // n
    print(f"(triangle, tile) pairs {npair}")
    steps = (span_s + 1) // 2
    # per pair: rows (segments incl. zero-span rows in the tile's row range are approximated by segments)
    prow = np.diff(brk)
    psteps_flat = np.add.reduceat(np.maximum(steps, 1), brk[:-1])
    # chunks: per tile, consecutive 64 pairs
    tb = np.r_[0, np.flatnonzero(np.diff(pair_tile)) + 1, npair]
    SETUP, SPAN, PIX = 200, 25, 40
    tot = {"nested": 0.0, "flat": 0.0, "ideal": 0.0, "setup": 0.0}
    nch = 0
    for t in range(len(tb) - 1):
        a, b = tb[t], tb[t + 1]
        for c0 in range(a, b, 64):
            c1 = min(c0 + 64, b)
            nch += 1
            tot["setup"] += SETUP
            # nested
            mr = prow[c0:c1].max()
            it = 0
            for k in range(mr):
                ms = 0
                for p in range(c0, c1):
                    if k < prow[p]:
                        ms = max(ms, steps[brk[p] + k])
                it += SPAN + PIX * ms
                tot["rowsteps"] = tot.get("rowsteps", 0) + 1
                tot["pixsteps"] = tot.get("pixsteps", 0) + ms
            tot["nested"] += it
            tot["flat"] += (SPAN + PIX) * psteps_flat[c0:c1].max()
            fr = span_s[brk[c0]:brk[c1]].sum()
            tot["ideal"] += PIX * math.ceil(fr / 128) + SPAN * math.ceil((brk[c1] - brk[c0]) / 64)
    print(f"chunks {nch}")
    for k, v in tot.items():
        print(f"{k:7s} {v / 1e6:8.2f} M wave-instr  per chunk {v / nch:8.1f}")


if __name__ == "__main__":
    main()
