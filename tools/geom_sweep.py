#!/usr/bin/env python3
"""Device-resident encode / reconstruct_into rates across code geometries
(planar batches, cold: two alternating batches, after 150 ms of untimed load).
Bytes: encode (d+p)*S per group, reconstruct (d+e)*S per group with e uniform
in [1, p] (every group lossy).  One JSON line per geometry."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ugo_amd import fec  # noqa: E402

GEOMS = [(10, 3, 1350), (5, 3, 1350), (8, 2, 1350), (12, 4, 1350), (16, 4, 1350), (20, 5, 1350),
         (24, 8, 1350), (32, 8, 9000), (40, 8, 2000), (48, 16, 1350)]
TARGET_BYTES = 1.2e9  # per batch, like the bench's 65,536 x (10+3) x 1360


def masks_for(G, n, p, gen):
    m = torch.full((G,), ((1 << n) - 1) if n < 64 else -1, dtype=torch.int64)
    e = torch.randint(1, p + 1, (G,), generator=gen)
    for g in range(G):
        for r in torch.randperm(n, generator=gen)[: int(e[g])].tolist():
            m[g] &= ~(1 << r) if r < 63 else (1 << 63) - 1
    return m.cuda(), e


def timed(fn, reps=20):
    t0 = time.time()
    while time.time() - t0 < 0.15:
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


def main():
    gen = torch.Generator().manual_seed(3)
    only = [tuple(int(x) for x in a.split(",")) for a in sys.argv[1:]]  # e.g. 48,16,1350
    for d, p, S in (only or GEOMS):
        n = d + p
        pitch = (S + 15) // 16 * 16
        G = max(256, int(TARGET_BYTES / (n * pitch)))
        enc = fec.New(d, p)
        bs = [torch.randint(0, 256, (n, G, pitch), dtype=torch.uint8, device="cuda") for _ in range(2)]
        outs = [torch.empty((p, G, pitch), dtype=torch.uint8, device="cuda") for _ in range(2)]
        masks, e = masks_for(G, n, p, gen)
        i = [0]

        def enc_step():
            enc.encode_batch(bs[i[0] & 1], S, shard_major=True)
            i[0] += 1

        def dec_step():
            k = i[0] & 1
            enc.reconstruct_into(bs[k], masks, outs[k], S, shard_major=True)
            i[0] += 1

        te = timed(enc_step)
        td = timed(dec_step)
        dec_bytes = float((d + e).sum()) * S
        print(json.dumps({"d": d, "p": p, "S": S, "groups": G,
                          "encode_us": round(te * 1e6, 1), "encode_TBps": round(G * n * S / te / 1e12, 3),
                          "reconstruct_into_us": round(td * 1e6, 1),
                          "reconstruct_into_TBps": round(dec_bytes / td / 1e12, 3)}), flush=True)
        del bs, outs


if __name__ == "__main__":
    main()
