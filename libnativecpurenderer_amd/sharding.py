"""Host-side helpers of the multi-GPU frame path.

Ownership rule (the same as the library's SetShard / owned_row): screen tile
row ty (32 pixel rows, nr_tri.h TH) belongs to shard ty % nshards.  These
helpers compute the owned rows/bands, assemble per-rank host arrays, and
bootstrap the RCCL communicator over an existing torch.distributed process
group (rank 0 creates the 128-byte id, every rank receives it).
"""
from __future__ import annotations

import numpy as np

TILE_H = 32


def band_pattern(nshards: int, slots=None):
    """Owner rank of each band slot; band b belongs to pattern[b % len(pattern)].
    Equal shards (slots None): 0..n-1 (SetShard).  Weighted: smooth weighted
    round robin over sum(slots) slots, lowest rank on ties (SetShardSlots,
    nr_dist.hip) -- the same integer algorithm, so host and device agree."""
    if slots is None:
        return list(range(nshards))
    slots = [int(v) for v in slots]
    period = sum(slots)
    credit = [0] * nshards
    out = []
    for _ in range(period):
        best = 0
        for p in range(nshards):
            credit[p] += slots[p]
            if credit[p] > credit[best]:
                best = p
        credit[best] -= period
        out.append(best)
    return out


def owned_bands(height: int, nshards: int, shard: int, tile_h: int = TILE_H, slots=None):
    """[(y0, y1), ...] half-open row ranges owned by `shard`."""
    pat = band_pattern(nshards, slots)
    bands = (height + tile_h - 1) // tile_h
    return [(b * tile_h, min(height, (b + 1) * tile_h)) for b in range(bands) if pat[b % len(pat)] == shard]


def owned_rows(height: int, nshards: int, shard: int, tile_h: int = TILE_H, slots=None) -> np.ndarray:
    rows = [np.arange(y0, y1) for y0, y1 in owned_bands(height, nshards, shard, tile_h, slots)]
    return np.concatenate(rows) if rows else np.zeros(0, dtype=np.int64)


def assemble(parts, height: int, nshards: int, tile_h: int = TILE_H, slots=None) -> np.ndarray:
    """parts[r] = rank r's full-size array, valid on its owned rows; returns
    the assembled frame (rows of each shard taken from its owner)."""
    out = np.empty_like(parts[0])
    for r, a in enumerate(parts):
        for y0, y1 in owned_bands(height, nshards, r, tile_h, slots):
            out[y0:y1] = a[y0:y1]
    return out


def broadcast_unique_id(dist, rank: int, make_uid) -> bytes:
    """The RCCL unique id of rank 0, on every rank of `dist`'s default group."""
    obj = [make_uid() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def make_comm(dist, world: int, rank: int):
    from . import libNativeCPURendererPybind as R
    uid = broadcast_unique_id(dist, rank, R.Comm.unique_id)
    return R.Comm(world, rank, uid)
