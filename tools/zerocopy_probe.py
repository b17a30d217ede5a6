#!/usr/bin/env python3
"""Host-path probe: reconstruct a pinned HOST batch in place with the device
kernels reading survivors and writing erased rows straight through PCIe
(zero-copy: the batch's device mapping), against the staged host path
(before zero-copy became ugo_fec_reconstruct_host's pinned path: H2D of whole
groups -> kernel -> erased rows back).
The zero-copy form moves d survivor rows in per group instead of all d+p.
Not product code."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ugo_amd import fec  # noqa: E402


def masks_uniform(G, n, emax, rng):
    m = np.empty(G, np.uint64)
    es = rng.integers(0, emax + 1, G)
    for g in range(G):
        m[g] = ((1 << n) - 1) & ~int(sum(1 << int(r) for r in rng.choice(n, int(es[g]), replace=False)))
    return m, es


def main():
    d, p, S, G, emax = 10, 3, 1350, 65536, 3
    if len(sys.argv) > 1 and sys.argv[1] == "jumbo":
        d, p, S, G, emax = 32, 8, 9000, 8192, 8
    n, pitch = d + p, (S + 15) // 16 * 16
    lib = fec.load_library()
    enc = fec.New(d, p)
    rng = np.random.default_rng(3)
    buf = fec.host_alloc(G * n * pitch)
    arr = buf.reshape(G, n, pitch)
    arr[:] = rng.integers(0, 256, (G, n, pitch), dtype=np.uint8)
    enc.encode_host(arr, S)
    want = arr.copy()
    masks, es = masks_uniform(G, n, emax, rng)
    dmask = torch.as_tensor(masks.view(np.int64)).cuda()
    st = torch.zeros(G, dtype=torch.int8, device="cuda")
    hip = ctypes.CDLL("libamdhip64.so")
    dptr = ctypes.c_void_p()
    assert hip.hipHostGetDevicePointer(ctypes.byref(dptr), ctypes.c_void_p(arr.ctypes.data), 0) == 0
    base = dptr.value  # the pinned batch's device mapping

    def zero_copy():
        rc = lib.ugo_fec_reconstruct_strided(enc._h, base, dmask.data_ptr(), G, S, pitch, n * pitch, 0,
                                             st.data_ptr(), None)
        assert rc == 0, rc

    res = {"case": f"({d}+{p})x{S} e~U[0,{emax}]", "groups": G}
    # staged host path (current ugo_fec_reconstruct_host)
    enc.reconstruct_host(arr, masks, S)
    t0 = time.perf_counter()
    for _ in range(3):
        enc.reconstruct_host(arr, masks, S)
    res["staged_ms"] = (time.perf_counter() - t0) / 3 * 1e3
    # zero-copy: kernels on the pinned batch
    for g in range(G):  # erase
        for r in range(n):
            if not (int(masks[g]) >> r) & 1:
                arr[g, r, :S] = 0
    zero_copy()
    torch.cuda.synchronize()
    res["zero_copy_bit_exact"] = bool(np.array_equal(arr[:, :, :S], want[:, :, :S])) and not st.any().item()
    t0 = time.perf_counter()
    for _ in range(3):
        zero_copy()
    torch.cuda.synchronize()
    res["zero_copy_ms"] = (time.perf_counter() - t0) / 3 * 1e3
    surv = G * d * S + int(es.sum()) * S
    res["zero_copy_pcie_GBps"] = surv / (res["zero_copy_ms"] * 1e-3) / 1e9
    # encode straight on the pinned batch too (d rows in, p rows out)
    def enc_zc():
        rc = lib.ugo_fec_encode_strided(enc._h, base, G, S, pitch, n * pitch, None)
        assert rc == 0, rc
    enc_zc()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        enc_zc()
    torch.cuda.synchronize()
    res["encode_zero_copy_ms"] = (time.perf_counter() - t0) / 3 * 1e3
    t0 = time.perf_counter()
    for _ in range(3):
        enc.encode_host(arr, S)
    res["encode_staged_ms"] = (time.perf_counter() - t0) / 3 * 1e3
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in res.items()}))
    fec.host_free(buf)


if __name__ == "__main__":
    main()
