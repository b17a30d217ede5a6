#!/usr/bin/env python3
"""Kernel-boundary cost of the bench step (encode -> reconstruct, 65,536 groups
of (10+3)x1350, planar): wall time per step with
  plain     -- ordinary launches (hipLaunchKernelGGL),
  timed     -- the launch-timing ABI on (hipExtLaunchKernel start/stop events),
  graph     -- K steps captured once into a HIP graph and replayed,
against the sum of the kernel durations (timing ABI).  Not product code."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ugo_amd import fec  # noqa: E402


def main():
    d, p, n, S, pitch, G, K = 10, 3, 13, 1350, 1360, 65536, 200
    enc = fec.New(d, p)
    gen = torch.Generator(device="cuda").manual_seed(1)
    sh = torch.randint(0, 256, (n, G, pitch), dtype=torch.uint8, device="cuda", generator=gen)
    rng = np.random.default_rng(2)
    m = np.empty(G, np.uint64)
    for g in range(G):
        a, b = rng.choice(n, 2, replace=False)
        m[g] = ((1 << n) - 1) & ~(1 << int(a)) & ~(1 << int(b))
    masks = torch.as_tensor(m.view(np.int64)).cuda()
    s = torch.cuda.current_stream()

    def step():
        enc.encode_batch(sh, S, stream=s, shard_major=True)
        enc.reconstruct_batch(sh, masks, S, stream=s, shard_major=True)

    def wall(fn, reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(reps)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps * 1e6

    for _ in range(60):
        step()
    res = {}
    res["plain_us_per_step"] = wall(lambda r: [step() for _ in range(r)], K)
    enc.timing_begin(4 * K + 16)
    res["timed_us_per_step"] = wall(lambda r: [step() for _ in range(r)], K)
    recs, _ = enc.timing_end()
    res["kernel_sum_us_per_step"] = float(recs["ms"].sum()) * 1e3 / K
    try:
        g = torch.cuda.CUDAGraph()
        cs = torch.cuda.Stream()
        cs.wait_stream(s)
        with torch.cuda.stream(cs):
            step()  # warm on the capture stream
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=cs):
            for _ in range(20):
                enc.encode_batch(sh, S, stream=cs, shard_major=True)
                enc.reconstruct_batch(sh, masks, S, stream=cs, shard_major=True)
        g.replay()
        torch.cuda.synchronize()
        res["graph_us_per_step"] = wall(lambda r: [g.replay() for _ in range(r // 20)], K)
    except Exception as e:  # noqa: BLE001
        res["graph_error"] = repr(e)[:200]
    res["plain_again_us_per_step"] = wall(lambda r: [step() for _ in range(r)], K)
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
