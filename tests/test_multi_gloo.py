"""World-size-2 CPU tests (gloo) of the multi-GPU frame orchestration:
tile-row ownership partitions the frame, per-rank owned rows gathered over
the process group reassemble the full frame byte for byte (rendered here by
the oracle, since there is no GPU), and the 128-byte communicator id rank 0
creates reaches every rank."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import scenes
from libnativecpurenderer_amd import sharding


def test_ownership_partitions_rows():
    for H in (1, 31, 32, 33, 1080, 2160):
        for n in (1, 2, 3, 8):
            rows = np.concatenate([sharding.owned_rows(H, n, r) for r in range(n)])
            assert np.array_equal(np.sort(rows), np.arange(H))
            # interleaved: the busy middle of a centred mesh is spread over all ranks
            if H >= 32 * n * 2:
                mid = [r for r in range(n) if any(y0 <= H // 2 < y1 or abs(y0 - H // 2) < 32 * n
                                                  for y0, y1 in sharding.owned_bands(H, n, r))]
                assert len(mid) == n


def test_weighted_band_patterns():
    """SetShardSlots' smooth weighted round robin (host restatement): every
    rank gets exactly slots[p] of each period, equal slots give SetShard's
    0..n-1, and a rank's bands are spread (no run longer than needed)."""
    assert sharding.band_pattern(4) == [0, 1, 2, 3]
    assert sharding.band_pattern(4, [1, 1, 1, 1]) == [0, 1, 2, 3]
    for slots in ([3, 1], [1, 4, 2], [6, 2, 2, 2, 2, 2, 2, 2], [10, 1, 1]):
        pat = sharding.band_pattern(len(slots), slots)
        assert len(pat) == sum(slots)
        assert [pat.count(p) for p in range(len(slots))] == slots
        big = max(range(len(slots)), key=lambda p: slots[p])
        run = max(len(x) for x in "".join("x" if q == big else " " for q in pat).split(" "))
        others = sum(slots) - slots[big]
        assert run <= -(-slots[big] // max(1, others)) + 1
    H = 2160
    for slots in ([3, 1], [6, 2, 2, 2, 2, 2, 2, 2]):
        n = len(slots)
        rows = np.concatenate([sharding.owned_rows(H, n, r, slots=slots) for r in range(n)])
        assert np.array_equal(np.sort(rows), np.arange(H))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        W, H = 120, 100
        xy, z, c = scenes.triangle_soup(500, W, H, 14, seed=5, gouraud=True)
        ctx = scenes.OracleFactory().context(W, H, False)
        ctx.set_color(0, 0, 0, 0)
        ctx.set_depth_state(True, True)
        ctx.clear_depth()
        ctx.draw_triangles(xy, c, z=z)
        full = ctx.get_buffer_numpy()
        mine = np.zeros_like(full)
        rows = sharding.owned_rows(H, world, rank)
        mine[rows] = full[rows]                      # what this rank owns
        parts = [None] * world
        dist.all_gather_object(parts, mine)
        asm = sharding.assemble(parts, H, world)
        uid = sharding.broadcast_unique_id(dist, rank, lambda: bytes(range(128)))
        q.put((rank, scenes.bits_equal(asm, full), uid == bytes(range(128))))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_assembly_and_id_broadcast():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert sorted(r[0] for r in res) == [0, 1]
    assert all(r[1] for r in res), res
    assert all(r[2] for r in res), res
