#!/usr/bin/env python3
"""RX from host memory: ugo_fec_rx_assemble reading a pinned packet ring over
PCIe (zero-copy, the library maps the ring) against H2D of the ring into
device memory + rx_assemble from there.  65,536 groups of (10+3), 5% loss,
1476-B packets in 1488-B slots, RC4 pad.  Checks both give the same batch.
Not product code."""
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
    d, p, n, S, pitch, slot, G = 10, 3, 13, 1470, 1472, 1488, 65536
    enc = fec.New(d, p)
    rng = np.random.default_rng(5)
    seq = np.arange(G * n, dtype=np.int64)
    seq = seq[rng.random(G * n) >= 0.05]
    rng.shuffle(seq)
    npk = seq.size
    ring = torch.empty((npk, slot), dtype=torch.uint8).pin_memory()
    ring.numpy()[:] = rng.integers(0, 256, (npk, slot), dtype=np.uint8)
    hdr = np.zeros((npk, 6), np.uint8)
    for b in range(4):
        hdr[:, b] = (seq >> (8 * b)) & 0xFF
    hdr[:, 4] = np.where(seq % n < d, 0xF1, 0xF2)
    ks = np.frombuffer(fec.rc4_keystream(b"1234567890123456", slot), np.uint8)
    ring.numpy()[:, :6] = hdr ^ ks[:6]
    lens_h = torch.full((npk,), 1476, dtype=torch.int16).pin_memory()
    pad = torch.from_numpy(ks.copy()).cuda()
    d_ring = torch.empty((npk, slot), dtype=torch.uint8, device="cuda")
    d_lens = torch.empty(npk, dtype=torch.int16, device="cuda")
    sh = [torch.zeros((n, G, pitch), dtype=torch.uint8, device="cuda") for _ in range(2)]
    pres = [torch.zeros(G, dtype=torch.int64, device="cuda") for _ in range(2)]
    s = torch.cuda.current_stream()

    def staged():
        d_ring.copy_(ring, non_blocking=True)
        d_lens.copy_(lens_h, non_blocking=True)
        pres[0].zero_()
        enc.rx_assemble(d_ring, d_lens, sh[0], pres[0], shard_size=S, pad=pad)

    def zero_copy():
        pres[1].zero_()
        enc.rx_assemble(ring, lens_h, sh[1], pres[1], shard_size=S, pad=pad)

    res = {"packets": int(npk), "ring_bytes": int(npk * slot)}
    for name, fn in (("staged", staged), ("zero_copy", zero_copy)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / 10
        res[f"{name}_ms"] = t * 1e3
        res[f"{name}_Mpkt_per_s"] = npk / t / 1e6
    res["same_batch"] = bool(torch.equal(sh[0][:, :, :S], sh[1][:, :, :S]) and torch.equal(pres[0], pres[1]))
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
