"""CPU model of the ordered raster's per-chunk load balance on C5 (round 6).

Per (triangle, 32x8 block) unit -- the triangle covers a pixel of the block (row spans by the ceil-crossing
rule, a band's union taken as one interval) -- grouped by tile, 64-entry chunk of the tile's ordered list
(tri_tiles' rectangle) and wave (block).  Reports sum over chunks of the most-loaded wave's units against
the mean wave's: the barrier per chunk makes every wave wait for the most-loaded one.
Usage: python tools/exp/c5_balance.py"""
import math
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0] + "/tests")
import scenes  # noqa: E402

W, H, TW, TH = 1920, 1080, 64, 32


def main():
    xy, z, c = scenes.triangle_soup(50000, W, H, 256.0, seed=1234, alpha=(0.2, 0.8))
    order = np.argsort(-z.mean(axis=1), kind="stable")
    xy = xy[order]
    n = len(xy)
    sx, sy = xy[:, 0::2], xy[:, 1::2]
    tx_n, ty_n = (W + TW - 1) // TW, (H + TH - 1) // TH
    # tile lists (tri_tiles): rows [ceil(ymin), ceil(ymax)), cols [floor(xmin)-2, ceil(xmax)+2]
    ymn, ymx = sy.min(1), sy.max(1)
    r0 = np.clip(np.ceil(ymn), 0, H).astype(int)
    r1 = np.clip(np.ceil(ymx), 0, H).astype(int)
    c0 = np.clip(np.floor(sx.min(1)) - 2, 0, W - 1).astype(int)
    c1 = np.clip(np.ceil(sx.max(1)) + 2, 0, W - 1).astype(int)
    pos = {}   # (tile) -> running count; per pair its chunk
    lists = [[] for _ in range(tx_n * ty_n)]
    for t in range(n):
        if r0[t] >= r1[t]:
            continue
        for ty in range(r0[t] // TH, (r1[t] - 1) // TH + 1):
            for tx in range(c0[t] // TW, c1[t] // TW + 1):
                lists[ty * tx_n + tx].append(t)
    chunk_of = {}
    for tile, L in enumerate(lists):
        for i, t in enumerate(L):
            chunk_of[(tile, t)] = i // 64
    # units: per triangle, per block row (8 rows), the union of its row spans
    units = {}
    for t in range(n):
        if r0[t] >= r1[t]:
            continue
        ys = np.arange(r0[t], r1[t], dtype=float)
        xs_l, xe_l = [], []
        for y in ys:
            cc = []
            for (i, j) in ((0, 2), (1, 0), (2, 1)):
                if (sy[t, i] > y) != (sy[t, j] > y):
                    cc.append((sx[t, j] - sx[t, i]) * (y - sy[t, i]) / (sy[t, j] - sy[t, i]) + sx[t, i])
            if len(cc) == 2:
                xs_l.append(min(max(math.ceil(min(cc)), 0), W))
                xe_l.append(min(max(math.ceil(max(cc)), 0), W))
            else:
                xs_l.append(0); xe_l.append(0)
        xs_a, xe_a = np.array(xs_l), np.array(xe_l)
        br = (ys // 8).astype(int)
        for b in np.unique(br):
            m = (br == b) & (xe_a > xs_a)
            if not m.any():
                continue
            a, e = xs_a[m].min(), xe_a[m].max()
            for bc in range(a // 32, (e - 1) // 32 + 1):
                tile = (b // 4) * tx_n + bc // 2
                wave = (b % 4) * 2 + bc % 2
                key = (tile, chunk_of[(tile, t)])
                units.setdefault(key, np.zeros(8, int))[wave] += 1
    mx = sum(v.max() for v in units.values())
    mean = sum(v.mean() for v in units.values())
    tot = sum(v.sum() for v in units.values())
    chunks = sum((len(L) + 63) // 64 for L in lists)
    print(f"units {tot}  chunks {chunks}  sum(max) {mx}  sum(mean) {mean:.0f}  ratio {mx / mean:.2f}")
    # per tile: max over waves of the tile's total (no barrier) vs sum over chunks of max
    per_tile = {}
    for (tile, ch), v in units.items():
        per_tile.setdefault(tile, np.zeros(8, int))
        per_tile[tile] += v
    tmx = sum(v.max() for v in per_tile.values())
    print(f"sum over tiles of the most-loaded wave's total (no per-chunk barrier): {tmx}  ratio to mean {tmx / mean:.2f}")


main()
