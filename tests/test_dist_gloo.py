"""CPU, world_size 2 over gloo: the N>1 path of bench.py.

Packet groups are independent codewords (ugo/fec.go:145-146), so ranks own
contiguous group ranges (ugo_amd.shard.partition) and no collective touches
the data path.  This test runs that decomposition on two processes with the
CPU oracle standing in for each rank's GPU (checker only), gathers the
per-rank outputs and checks they equal the single-process result, and checks
the max-over-ranks timing reduction bench.py uses.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ugo_amd.shard import partition


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "oracle"))
    import rs_ref

    d, p, S = 10, 3, 64
    n = d + p
    g0, g1 = partition(total, world, rank)
    rng = np.random.default_rng(123)
    full = rng.integers(0, 256, (total, n, S), dtype=np.uint8)  # same synthetic batch on every rank
    mine = np.ascontiguousarray(full[g0:g1])
    rs_ref.c_encode(d, p, mine)
    masks = np.full(g1 - g0, ((1 << n) - 1) & ~(1 << 2) & ~(1 << 11), np.uint64)
    erased = mine.copy()
    erased[:, [2, 11]] = 0
    rs_ref.c_reconstruct(d, p, erased, masks)
    ok = np.array_equal(erased, mine)
    # gather every rank's encoded slice (only to check coverage; bench.py never does this)
    sizes = [partition(total, world, r)[1] - partition(total, world, r)[0] for r in range(world)]
    buf = torch.zeros((max(sizes), n, S), dtype=torch.uint8)
    buf[: g1 - g0] = torch.from_numpy(mine)
    gathered = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(gathered, buf)
    t = torch.tensor([0.5 + rank], dtype=torch.float64)  # per-rank elapsed
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    okt = torch.tensor([int(ok)])
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    if rank == 0:
        merged = np.concatenate([gathered[r][: sizes[r]].numpy() for r in range(world)])
        ref = full.copy()
        rs_ref.c_encode(d, p, ref)
        out_q.put((bool(np.array_equal(merged, ref)), float(t.item()), bool(okt.item())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("total", [1000, 7])
def test_two_rank_sharding_matches_single_process(total):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, total, q)) for r in range(2)]
    for pr in procs:
        pr.start()
    res = q.get(timeout=120)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    same, tmax, ok = res
    assert same, "concatenated per-rank results differ from the single-process encode"
    assert tmax == 1.5, "max-over-ranks timing reduction"
    assert ok


def test_partition_covers_exactly_once():
    for total in (0, 1, 7, 65536, 4194304):
        for world in (1, 2, 3, 8):
            ranges = [partition(total, world, r) for r in range(world)]
            assert ranges[0][0] == 0 and ranges[-1][1] == total
            for (a0, a1), (b0, b1) in zip(ranges, ranges[1:]):
                assert a1 == b0 and a0 <= a1
            sizes = [b - a for a, b in ranges]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        partition(10, 2, 2)
