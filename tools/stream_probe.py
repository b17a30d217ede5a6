#!/usr/bin/env python3
"""Bench-step probe: K steps of encode + reconstruct over 2 alternating batches,
on one stream (the bench) vs steps alternating between two streams (step k on
stream k % 2, so consecutive steps -- independent batches -- may overlap at
their kernel boundaries).  Not product code."""
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
    bat = [torch.randint(0, 256, (n, G, pitch), dtype=torch.uint8, device="cuda", generator=gen) for _ in range(2)]
    rng = np.random.default_rng(2)
    m = np.empty(G, np.uint64)
    for g in range(G):
        a, b = rng.choice(n, 2, replace=False)
        m[g] = ((1 << n) - 1) & ~(1 << int(a)) & ~(1 << int(b))
    masks = torch.as_tensor(m.view(np.int64)).cuda()
    s0 = torch.cuda.current_stream()
    s1 = torch.cuda.Stream()
    streams = [s0, s1]

    def run(two):
        for k in range(K):
            s = streams[k % 2] if two else s0
            b = bat[k % 2]
            enc.encode_batch(b, S, stream=s, shard_major=True)
            enc.reconstruct_batch(b, masks, S, stream=s, shard_major=True)

    res = {}
    for name, two in (("one_stream", False), ("two_streams", True), ("one_stream_again", False)):
        run(two)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(two)
        torch.cuda.synchronize()
        res[name + "_us_per_step"] = (time.perf_counter() - t0) / K * 1e6
    print(json.dumps({k: round(v, 2) for k, v in res.items()}))


if __name__ == "__main__":
    main()
