#!/usr/bin/env python3
"""Host-buffer (PCIe-inclusive) and jumbo-geometry measurements for DESIGN.md.

BASELINE configs[4]: (32+8)x9000 B groups, mixed erasure patterns
(e uniform in 0..8, positions uniform among the 40 shards), timed with the
pinned hipMemcpyAsync H2D/D2H included.  The same host path is also measured
for the (10+3)x1350 geometry, and the jumbo geometry device-resident.

The host path is ugo_fec_encode_host / ugo_fec_reconstruct_host: the engine
chunks the batch over 3 internal streams (H2D -> kernel -> D2H per chunk).
Bytes reported are the algorithmic bytes of BASELINE.md ((d+p)*S encode,
(d+e)*S reconstruct); "pcie_bytes" counts what actually crosses the link.
Prints one JSON object per measurement.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ugo_amd import fec  # noqa: E402


def masks_mixed(G, n, emax, rng):
    m = np.full(G, (1 << n) - 1, np.uint64)
    es = rng.integers(0, emax + 1, G)
    for g in range(G):
        for r in rng.choice(n, int(es[g]), replace=False):
            m[g] &= ~np.uint64(1 << int(r))
    return m, es


def warm(fn, ms=150.0):
    """Run fn back to back for `ms` of wall time: the clocks take ~20 ms of
    load to reach steady state, so a few untimed calls measure the ramp."""
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(10):
            fn()
        torch.cuda.synchronize()


def host_case(d, p, S, G, emax, reps, pinned=True):
    n = d + p
    pitch = (S + 15) // 16 * 16
    enc = fec.New(d, p)
    nbytes = G * n * pitch
    rng = np.random.default_rng(7)
    if pinned:
        raw = fec.host_alloc(nbytes)
        arr = raw.reshape(G, n, pitch)
    else:
        arr = np.empty((G, n, pitch), np.uint8)
    arr[:] = rng.integers(0, 256, (G, n, pitch), dtype=np.uint8)
    masks, es = masks_mixed(G, n, emax, rng)
    enc.encode_host(arr, S)  # warm up (allocates staging)
    t0 = time.perf_counter()
    for _ in range(reps):
        enc.encode_host(arr, S)
    t_enc = (time.perf_counter() - t0) / reps
    keep = arr.copy()
    st = np.zeros(G, np.int8)
    enc.reconstruct_host(arr, masks, S, status=st)
    t0 = time.perf_counter()
    for _ in range(reps):
        enc.reconstruct_host(arr, masks, S, status=st)
    t_dec = (time.perf_counter() - t0) / reps
    ok = bool(np.array_equal(arr[:, :, :S], keep[:, :, :S])) and not st.any()
    alg_enc = G * n * S
    alg_dec = int(sum(d + int(e) for e in es if int(e) > 0) * S)  # a group with no erasure moves nothing
    # pinned: zero-copy -- the kernels read d survivor rows per group and write the erased rows over PCIe;
    # pageable: staged -- whole groups in, whole groups out; + masks and statuses either way
    # (zero-copy reads nothing for a group with no erasure)
    e_rows = int(sum(int(e) for e in es))
    lossy = int(sum(1 for e in es if int(e) > 0))
    dec_pcie = (lossy * d * S + e_rows * S if pinned else 2 * G * n * pitch) + 9 * G
    out = [
        {"case": f"host encode ({d}+{p})x{S}", "groups": G, "pinned": pinned, "ms": t_enc * 1e3,
         "alg_GBps": alg_enc / t_enc / 1e9, "pcie_bytes": G * (d * pitch + p * S),
         "pcie_GBps": G * (d * pitch + p * S) / t_enc / 1e9},
        {"case": f"host reconstruct ({d}+{p})x{S} e~U[0,{emax}]", "groups": G, "pinned": pinned,
         "ms": t_dec * 1e3, "alg_GBps": alg_dec / t_dec / 1e9, "pcie_bytes": dec_pcie,
         "pcie_GBps": dec_pcie / t_dec / 1e9, "round_trip_ok": ok},
    ]
    if pinned:
        fec.host_free(raw)
    return out


def device_case(d, p, S, G, emax, reps):
    n = d + p
    pitch = (S + 15) // 16 * 16
    enc = fec.New(d, p)
    sh = torch.randint(0, 256, (n, G, pitch), dtype=torch.uint8, device="cuda")
    rng = np.random.default_rng(9)
    masks, es = masks_mixed(G, n, emax, rng)
    dm = torch.as_tensor(masks.view(np.int64)).cuda()
    s = torch.cuda.current_stream()
    def both():
        enc.encode_batch(sh, S, shard_major=True)
        enc.reconstruct_batch(sh, dm, S, shard_major=True)
    warm(both)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    e[0].record(s)
    for _ in range(reps):
        enc.encode_batch(sh, S, shard_major=True)
    e[1].record(s)
    for _ in range(reps):
        enc.reconstruct_batch(sh, dm, S, shard_major=True)
    e[2].record(s)
    out = torch.empty((p, G, pitch), dtype=torch.uint8, device="cuda")
    ei = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ei[0].record(s)
    for _ in range(reps):
        enc.reconstruct_into(sh, dm, out, S, shard_major=True)
    ei[1].record(s)
    torch.cuda.synchronize()
    te = e[0].elapsed_time(e[1]) / reps * 1e-3
    td = e[1].elapsed_time(e[2]) / reps * 1e-3
    ti = ei[0].elapsed_time(ei[1]) / reps * 1e-3
    alg_dec = int(sum(d + int(x) for x in es if int(x) > 0) * S)  # a group with no erasure moves nothing
    return [{"case": f"device encode ({d}+{p})x{S}", "groups": G, "us": te * 1e6, "alg_GBps": G * n * S / te / 1e9},
            {"case": f"device reconstruct ({d}+{p})x{S} e~U[0,{emax}]", "groups": G, "us": td * 1e6,
             "alg_GBps": alg_dec / td / 1e9},
            {"case": f"device reconstruct_into ({d}+{p})x{S} e~U[0,{emax}]", "groups": G, "us": ti * 1e6,
             "alg_GBps": alg_dec / ti / 1e9}]


def rx_case(G, loss, reps, encrypt=True):
    """RX path device-resident: packets already in HBM (16-B slots of 1488 B),
    RC4 pad XOR + header decode + planar placement (ugo_fec_rx_assemble), then
    data-only Reconstruct of the batch.  Synthetic payloads (not codewords:
    throughput only; parity is covered by tests/test_rx_batch.py)."""
    d, p, n, S, pitch, slot = 10, 3, 13, 1470, 1472, 1488
    enc = fec.New(d, p)
    gen = torch.Generator(device="cuda").manual_seed(3)
    seq = torch.arange(G * n, device="cuda", dtype=torch.int64)
    keep = torch.rand(G * n, device="cuda", generator=gen) >= loss
    seq = seq[keep]
    seq = seq[torch.randperm(seq.numel(), device="cuda", generator=gen)]
    npk = seq.numel()
    wire = torch.randint(0, 256, (npk, slot), dtype=torch.uint8, device="cuda", generator=gen)
    hdr = torch.zeros((npk, 6), dtype=torch.uint8, device="cuda")
    for b in range(4):
        hdr[:, b] = ((seq >> (8 * b)) & 0xFF).to(torch.uint8)
    hdr[:, 4] = torch.where(seq % n < d, 0xF1, 0xF2).to(torch.uint8)
    pad = torch.frombuffer(bytearray(fec.rc4_keystream(b"1234567890123456", slot)), dtype=torch.uint8).cuda()
    if encrypt:
        hdr ^= pad[:6]
    wire[:, :6] = hdr
    lens = torch.full((npk,), 1476, dtype=torch.int16, device="cuda")
    sh = torch.empty((n, G, pitch), dtype=torch.uint8, device="cuda")
    present = torch.zeros(G, dtype=torch.int64, device="cuda")
    st = torch.zeros(5, dtype=torch.int32, device="cuda")

    def run():
        present.zero_()
        enc.rx_assemble(wire, lens, sh, present, shard_size=S, pad=pad if encrypt else None, stats=st)
        enc.reconstruct_batch(sh, present, shard_size=S, data_only=True, shard_major=True)

    warm(run)
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    s = torch.cuda.current_stream()
    e[0].record(s)
    for _ in range(reps):
        present.zero_()
        enc.rx_assemble(wire, lens, sh, present, shard_size=S, pad=pad if encrypt else None, stats=st)
    e[1].record(s)
    for _ in range(reps):
        enc.reconstruct_batch(sh, present, shard_size=S, data_only=True, shard_major=True)
    e[2].record(s)
    out = torch.empty((p, G, pitch), dtype=torch.uint8, device="cuda")
    ei = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ei[0].record(s)
    for _ in range(reps):
        enc.reconstruct_into(sh, present, out, shard_size=S, data_only=True, shard_major=True)
    ei[1].record(s)
    torch.cuda.synchronize()
    ta = e[0].elapsed_time(e[1]) / reps * 1e-3
    tr = e[1].elapsed_time(e[2]) / reps * 1e-3
    ti = ei[0].elapsed_time(ei[1]) / reps * 1e-3
    # per-kernel durations of rx_assemble: optimistic placement, then the three
    # dedupe kernels gated on the duplicate flag (empty launches without duplicates)
    names = ("place", "claim_fill_gated", "claim_gated", "replace_gated")
    enc.timing_begin(len(names) * reps)
    for _ in range(reps):
        present.zero_()
        enc.rx_assemble(wire, lens, sh, present, shard_size=S, pad=pad if encrypt else None, stats=st)
    recs, _ = enc.timing_end()
    ms = recs["ms"].reshape(-1, len(names))
    kern = {nm: round(float(np.median(ms[:, k])) * 1e3, 1) for k, nm in enumerate(names)}
    asm_bytes = npk * (1476 + S)  # packet read + slot write
    return [{"case": f"rx assemble (10+3) loss={loss} rc4={encrypt}", "groups": G, "packets": npk,
             "us": ta * 1e6, "GBps": asm_bytes / ta / 1e9, "Mpkt_per_s": npk / ta / 1e6, "kernel_us": kern},
            {"case": f"rx reconstruct data-only after assemble", "groups": G, "us": tr * 1e6,
             "Mpkt_per_s_total": npk / (ta + tr) / 1e6},
            {"case": f"rx reconstruct_into data-only after assemble", "groups": G, "us": ti * 1e6,
             "Mpkt_per_s_total": npk / (ta + ti) / 1e6}]


def tx_case(G, reps, encrypt=True, full=True, d=10, p=3, max_len=1476):
    """TX path device-resident (ugo_fec_tx_assemble): G groups of d outgoing
    data packets (16-B slots) -> headers + parity over [6, maxsize) + RC4 pad
    XOR -> d+p wire packets per group.  Bytes = packet bytes read + wire bytes
    written."""
    n, slot = d + p, (max_len + 15) // 16 * 16
    enc = fec.New(d, p)
    gen = torch.Generator(device="cuda").manual_seed(5)
    pk = torch.randint(0, 256, (G * d, slot), dtype=torch.uint8, device="cuda", generator=gen)
    if full:
        lens = torch.full((G * d,), max_len, dtype=torch.int16, device="cuda")
    else:
        lens = torch.randint(6, max_len + 1, (G * d,), dtype=torch.int16, device="cuda", generator=gen)
    wire = torch.empty((G * n, slot), dtype=torch.uint8, device="cuda")
    wl = torch.empty(G * n, dtype=torch.int16, device="cuda")
    pad = torch.frombuffer(bytearray(fec.rc4_keystream(b"1234567890123456", slot)), dtype=torch.uint8).cuda()
    run = lambda: enc.tx_assemble(pk, lens, wire, wl, pad=pad if encrypt else None, max_len=max_len)  # noqa: E731
    warm(run)
    s = torch.cuda.current_stream()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record(s)
    for _ in range(reps):
        run()
    e[1].record(s)
    torch.cuda.synchronize()
    t = e[0].elapsed_time(e[1]) / reps * 1e-3
    L = lens.to(torch.int64).view(G, d)
    moved = int(2 * L.sum().item() + p * L.max(dim=1).values.sum().item())
    return [{"case": f"tx assemble ({d}+{p})x{max_len} full={full} rc4={encrypt}", "groups": G, "packets_out": G * n,
             "us": t * 1e6, "GBps": moved / t / 1e9, "Mpkt_per_s": G * n / t / 1e6}]


def _uvarint_np(v, nbytes):
    """v (uint64 array) as fixed-width uvarints of nbytes (continuation bits set)."""
    out = np.zeros((v.size, nbytes), np.uint8)
    for j in range(nbytes):
        out[:, j] = ((v >> np.uint64(7 * j)) & np.uint64(0x7F)).astype(np.uint8)
        if j < nbytes - 1:
            out[:, j] |= 0x80
    return out


def pkt_case(npk, reps, ack_frac=0.25):
    """Wire-codec decode (ugo_fec_packet_decode) of a batch of received,
    FEC-framed, RC4-encrypted ugo data packets: 6-B FEC header, flags (PSH, a
    quarter with a SACK), 3-byte packet number, one segment (4-byte offset,
    BE16 length, 1400 data bytes).  Synthetic; parity is tests/test_packet_codec.py."""
    slot = 1488
    rng = np.random.default_rng(11)
    host = rng.integers(0, 256, (npk, slot), dtype=np.uint8)
    seq = np.arange(npk, dtype=np.uint64)
    host[:, 0:4] = seq.astype("<u4").view(np.uint8).reshape(npk, 4)
    host[:, 4] = 0xF1
    host[:, 5] = 0
    ack = rng.random(npk) < ack_frac
    pos = np.full(npk, 6)
    host[:, 6] = np.where(ack, 0xA0, 0x20)
    pos += 1
    # SACK without missing ranges: type 0, largest (3 B), delay (2 B), first block length (1 B)
    sack = np.concatenate([np.zeros((npk, 1), np.uint8), _uvarint_np(seq + np.uint64(1 << 15), 3),
                           np.full((npk, 2), 7, np.uint8), np.full((npk, 1), 5, np.uint8)], axis=1)
    rows = np.nonzero(ack)[0]
    host[rows[:, None], 7 + np.arange(7)[None, :]] = sack[rows]
    pos[ack] += 7
    pn = _uvarint_np(seq + np.uint64(1 << 15), 3)
    seg = np.concatenate([_uvarint_np(seq * np.uint64(1400), 4),
                          np.tile(np.array([[1400 >> 8, 1400 & 0xFF]], np.uint8), (npk, 1))], axis=1)
    hdr = np.concatenate([pn, seg], axis=1)  # 9 bytes
    for j in range(9):
        host[np.arange(npk), pos + j] = hdr[:, j]
    lens = (pos + 9 + 1400).astype(np.int16)
    ks = np.frombuffer(fec.rc4_keystream(b"1234567890123456", slot), np.uint8)
    host ^= ks[None, :]
    enc = fec.New(10, 3)
    d_pk = torch.from_numpy(host).cuda()
    d_len = torch.from_numpy(lens).cuda()
    pad = torch.from_numpy(ks.copy()).cuda()
    bufs = enc.packet_decode(d_pk, d_len, pad=pad, framed=True, max_ranges=4, max_segments=2)
    info = bufs[0]
    torch.cuda.synchronize()
    st = info.cpu().numpy().view(fec.PKT_INFO_DTYPE).reshape(-1)
    assert (st["status"] == 0).all() and (st["n_segments"] == 1).all(), "synthetic packets must decode"
    warm(lambda: enc.packet_decode(d_pk, d_len, pad=pad, framed=True, max_ranges=4, max_segments=2, out=bufs))
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    s = torch.cuda.current_stream()
    e[0].record(s)
    for _ in range(reps):
        enc.packet_decode(d_pk, d_len, pad=pad, framed=True, max_ranges=4, max_segments=2, out=bufs)
    e[1].record(s)
    torch.cuda.synchronize()
    t = e[0].elapsed_time(e[1]) / reps * 1e-3
    return [{"case": "packet decode (FEC-framed, RC4, 1 segment, 25% SACK)", "packets": npk, "us": t * 1e6,
             "Mpkt_per_s": npk / t / 1e6, "out_bytes_per_pkt": 64 + 4 * 16 + 2 * 16}]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    res = []
    if args.only == "txjumbo":
        for r in tx_case(8192, args.reps, d=32, p=8, max_len=9006):
            print(json.dumps(r), flush=True)
        return
    if args.only == "jumbo":
        for r in device_case(32, 8, 9000, 8192, 8, args.reps):
            print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()}))
        return
    if args.only == "host":
        res = host_case(32, 8, 9000, 8192, 8, args.reps, pinned=True)
        res += host_case(10, 3, 1350, 65536, 3, args.reps, pinned=True)
        res += host_case(10, 3, 1350, 65536, 3, 2, pinned=False)
        for r in res:
            print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()}))
        return
    if args.only == "pkt":
        for r in pkt_case(851968, args.reps):
            print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()}))
        return
    res += tx_case(65536, args.reps)
    res += tx_case(65536, args.reps, full=False)
    res += tx_case(65536, args.reps, encrypt=False)
    if args.only == "tx":
        for r in res:
            print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()}))
        return
    res += rx_case(65536, 0.05, args.reps)
    res += rx_case(65536, 0.05, args.reps, encrypt=False)
    if args.only == "rx":
        for r in res:
            print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()}))
        return
    res += device_case(32, 8, 9000, 8192, 8, args.reps)
    res += host_case(32, 8, 9000, 8192, 8, args.reps, pinned=True)
    res += host_case(10, 3, 1350, 65536, 3, args.reps, pinned=True)
    res += host_case(10, 3, 1350, 65536, 3, 2, pinned=False)
    for r in res:
        print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()}))


if __name__ == "__main__":
    main()
