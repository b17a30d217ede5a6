"""torchrun target for tests/test_bench_dist.py (CPU, gloo): one rank of
bench.py's multi-GPU decomposition with the CPU oracle standing in for the
rank's GPU (checker only).  It calls bench.py's own coordination functions --
dist_setup, rank_groups, clock_warmup, timed_region, reduce_max, all_ranks_ok
-- and rank 0 prints one JSON result line, as bench.py's ranks do."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import bench  # noqa: E402
import rs_ref  # noqa: E402


def main():
    total = int(os.environ.get("BENCH_TEST_TOTAL", "1000"))
    args = bench.parse(sys.argv[1:])
    rank, local_rank, world = bench.dist_setup("gloo")
    assert world == args.gpus, (world, args.gpus)
    d, p, S = 10, 3, 64
    n = d + p
    g0, G, scaling, tot = bench.rank_groups(total, 0, rank, world)
    rng = np.random.default_rng(123)
    full = rng.integers(0, 256, (total, n, S), dtype=np.uint8)  # same synthetic batch on every rank
    mine = np.ascontiguousarray(full[g0:g0 + G])
    ref = full.copy()
    rs_ref.c_encode(d, p, ref)

    def step():
        rs_ref.c_encode(d, p, mine)

    cw_ms, cw_steps, settled = bench.clock_warmup(step, lambda: None, 5.0)
    elapsed = bench.timed_region(step, 3, lambda: None, world)
    ok = bool(np.array_equal(mine, ref[g0:g0 + G]))
    erased = mine.copy()
    erased[:, [2, 11]] = 0
    masks = np.full(G, ((1 << n) - 1) & ~(1 << 2) & ~(1 << 11), np.uint64)
    rs_ref.c_reconstruct(d, p, erased, masks)
    ok = ok and bool(np.array_equal(erased, mine))
    # host-path coordination (bench.host_path_leg): NUMA placement from a fake
    # sysfs, barrier-started reps timed as max over ranks, summed bytes
    host = None
    sysfs = os.environ.get("BENCH_TEST_SYSFS")
    if sysfs:
        from ugo_amd import numa

        bdf = ["0000:0b:00.0", "0000:8c:00.0"][rank % 2]
        place = numa.gpu_numa_node(rank, sysfs=sysfs, bdf=bdf)
        saved = os.sched_getaffinity(0)
        bound = numa.bind_to_node(place)
        now = sorted(os.sched_getaffinity(0))
        os.sched_setaffinity(0, saved)
        import time

        t_job, t_mine = bench.timed_reps(lambda: time.sleep(0.01 * (1 + 2 * rank)), 3, world)
        total_bytes = bench.reduce_sum([1000 * (rank + 1)], world)[0]
        placement = bench.gather_objects({"rank": rank, "numa_node": place["numa_node"], "cpus": now,
                                          "bound": bound["bound"]}, world)
        host = {"t_job": t_job, "t_mine": t_mine, "bytes": total_bytes, "placement": placement}
    # rx_tx on every rank (bench.rx_tx_over_ranks): rank 0's leg + the max of each kernel time
    leg = {"rx_in_order": {"rx_assemble_ms": 0.4 + rank, "stats": [1, 2]}, "tx": {"tx_assemble_ms": 0.3 - 0.1 * rank},
           "note": "x"}
    rxtx = bench.rx_tx_over_ranks(leg, bench.gather_objects(leg, world))
    tmax, gmax, ranks = bench.reduce_max([0.5 + rank, G, rank], world)
    covered = bench.reduce_max([g0 + G if rank == world - 1 else 0], world)[0]
    all_ok = bench.all_ranks_ok(ok, world)
    one_bad = bench.all_ranks_ok(ok and rank != world - 1, world)
    if rank == 0:
        print(json.dumps({"metric": "test", "n_gpus": world, "scaling": scaling, "total_groups": tot,
                          "tmax": tmax, "gmax": gmax, "max_rank": ranks, "covered": covered, "all_ok": all_ok,
                          "one_bad": one_bad, "elapsed_pos": elapsed > 0, "cw_steps": cw_steps, "host": host,
                          "rx_tx": rxtx}),
              flush=True)
    else:
        print("rank %d noise on stdout" % rank, flush=True)
    import torch.distributed as dist

    dist.destroy_process_group()


if __name__ == "__main__":
    main()
