"""Distinct contexts on distinct host threads run concurrently (SURVEY.md §8b,
threading: "one context per device; calls on one context are serialised by the
caller; distinct contexts can run concurrently from different threads").

Four threads, each with its own context and its own HIP stream -- two on the
headline (10,3) code (host-built descriptor table), one on the jumbo (32,8) code
(per-group descriptors from stream-ordered scratch, k_prepare + k_apply_q) and
one on the per-group host path (pinned zero-copy reconstruct) -- loop encode and
reconstruct at the same time (ctypes releases the GIL inside every call).
Every thread's final bytes must equal the CPU oracle's (checker only)."""
import threading

import numpy as np
import pytest
import torch

import rs_ref
from ugo_amd import fec


def _masks(G, n, emax, rng):
    m = np.full(G, (1 << n) - 1, np.uint64)
    for g in range(G):
        for r in rng.choice(n, int(rng.integers(0, emax + 1)), replace=False):
            m[g] &= ~np.uint64(1 << int(r))
    return m


def _device_worker(d, p, S, G, iters, seed, out, key):
    n = d + p
    pitch = (S + 15) // 16 * 16
    rng = np.random.default_rng(seed)
    host = rng.integers(0, 256, (G, n, pitch), dtype=np.uint8)
    masks = _masks(G, n, p, rng)
    enc = fec.New(d, p)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        t = torch.as_tensor(np.ascontiguousarray(host.transpose(1, 0, 2))).cuda()
        dm = torch.as_tensor(masks.view(np.int64)).cuda()
        outb = torch.zeros((p, G, pitch), dtype=torch.uint8, device="cuda")
        for _ in range(iters):
            enc.encode_batch(t, S, stream=s, shard_major=True)
            enc.reconstruct_into(t, dm, outb, S, stream=s, shard_major=True)
    s.synchronize()
    out[key] = (host, masks, t.cpu().numpy().transpose(1, 0, 2), outb.cpu().numpy().transpose(1, 0, 2))


def _host_worker(d, p, S, iters, seed, out, key):
    rng = np.random.default_rng(seed)
    enc = fec.New(d, p)
    results = []
    for _ in range(iters):
        shards = [bytearray(rng.integers(0, 256, S, dtype=np.uint8).tobytes()) for _ in range(d)]
        shards += [bytearray(S) for _ in range(p)]
        enc.Encode(shards)
        full = [bytes(x) for x in shards]
        lost = rng.choice(d + p, p, replace=False)
        for r in lost:
            shards[int(r)] = None
        enc.Reconstruct(shards)
        results.append((full, [bytes(x) for x in shards]))
    out[key] = results


@pytest.mark.gpu
def test_contexts_on_threads_run_concurrently(gpu):
    out, errs = {}, []

    def guard(fn, *a):
        try:
            fn(*a)
        except BaseException as e:  # surfaced below, with the thread's name
            errs.append((a[-1], repr(e)))

    ths = [threading.Thread(target=guard, args=(_device_worker, 10, 3, 1350, 4096, 12, 1, out, "a")),
           threading.Thread(target=guard, args=(_device_worker, 10, 3, 1350, 2048, 12, 2, out, "b")),
           threading.Thread(target=guard, args=(_device_worker, 32, 8, 9000, 96, 6, 3, out, "jumbo")),
           threading.Thread(target=guard, args=(_host_worker, 10, 3, 1476, 40, 4, out, "host"))]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=300)
    assert not errs, errs
    for key, d, p, S in (("a", 10, 3, 1350), ("b", 10, 3, 1350), ("jumbo", 32, 8, 9000)):
        host, masks, got, outb = out[key]
        n = d + p
        want = host.copy()
        rs_ref.c_encode(d, p, want, S=S)
        assert np.array_equal(got[:, :, :S], want[:, :, :S]), f"{key}: encode"
        for g in range(0, host.shape[0], 7):  # a sample of groups: outputs = erased rows, ascending
            er = [r for r in range(n) if not (int(masks[g]) >> r) & 1]
            if len(er) > p:
                continue
            for i, r in enumerate(er):
                assert np.array_equal(outb[g, i, :S], want[g, r, :S]), f"{key}: group {g} output {i}"
    for full, rec in out["host"]:
        assert rec == full, "host path: reconstructed shards"


@pytest.mark.gpu
def test_host_paths_on_threads_share_the_copy_stream(gpu):
    """Round 6: every context's host-path H2D copies go to the ONE low-priority
    copy stream of the device (the process's hardware-queue budget).  Three
    threads, each with its own context, run host TX, host RX and the staged
    encode at the same time, three calls each, and every result equals the
    device-resident path's (host TX, host RX -- themselves checked against the
    sender loop and fec_ref + rs_ref in test_tx_batch / test_rx_batch) or the
    oracle's (staged encode) -- the shared stream orders the contexts' copies
    but never mixes their bytes or waits."""
    d, p, n, slot, L = 10, 3, 13, 1488, 1476
    S = L - 6
    G = 3000
    dev = torch.device("cuda")
    gen = torch.Generator(device=dev).manual_seed(61)
    pad = fec.rc4_keystream(b"1234567890123456", slot)
    dpad = torch.frombuffer(bytearray(pad), dtype=torch.uint8).to(dev)
    ref = fec.New(d, p)
    # TX inputs and the device path's wire packets
    dp = torch.randint(0, 256, (G * d, slot), dtype=torch.uint8, device=dev, generator=gen)
    tl = torch.full((G * d,), L, dtype=torch.int16, device=dev)
    dw = torch.empty((G * n, slot), dtype=torch.uint8, device=dev)
    dwl = torch.empty(G * n, dtype=torch.int16, device=dev)
    ref.tx_assemble(dp, tl, dw, dwl, pad=dpad, max_len=L)
    # RX: those wire packets minus 5 %, shuffled; the device path's recovered rows
    keep = torch.rand(G * n, device=dev, generator=gen) >= 0.05
    idx = torch.nonzero(keep).flatten()
    idx = idx[torch.randperm(idx.numel(), device=dev, generator=gen)]
    ring_d = dw[idx].contiguous()
    rl = torch.full((idx.numel(),), L, dtype=torch.int16, device=dev)
    bat = torch.empty((n, G, 1536), dtype=torch.uint8, device=dev)
    pr = torch.zeros(G, dtype=torch.int64, device=dev)
    ref.rx_assemble(ring_d, rl, bat, pr, shard_size=S, pad=dpad, frames=True)
    rows = torch.empty((G * p, 1536), dtype=torch.uint8, device=dev)
    rix = torch.empty(G * p, dtype=torch.int32, device=dev)
    cnt = ref.recover_data(bat, pr, rows, rix, shard_size=S + 6)
    torch.cuda.synchronize()
    k = int(cnt.item())
    want_rx = (rix[:k].cpu().numpy().astype(np.uint32), rows[:k, 6:6 + S].cpu().numpy())
    want_tx = (dw.cpu().numpy(), dwl.cpu().numpy().view(np.uint16))
    # staged encode (pageable, >= 3 chunks of the 64-MiB stage)
    rng = np.random.default_rng(62)
    host_enc = rng.integers(0, 256, (8000, n, 1360), dtype=np.uint8)
    want_enc = host_enc.copy()
    rs_ref.c_encode(d, p, want_enc, S=1350)
    bufs, errs, got = [], [], {}

    def pinned(shape, dtype=np.uint8):
        a = fec.host_alloc(int(np.prod(shape)) * np.dtype(dtype).itemsize).view(dtype).reshape(shape)
        bufs.append(a)
        return a

    pk, pl = pinned((G * d, slot)), pinned((G * d,), np.uint16)
    pk[:] = dp.cpu().numpy()
    pl[:] = L
    ring, rlens = pinned((idx.numel(), slot)), pinned((idx.numel(),), np.uint16)
    ring[:] = ring_d.cpu().numpy()
    rlens[:] = L
    wire, wl = pinned((G * n, slot)), pinned((G * n,), np.uint16)

    def tx():
        enc = fec.New(d, p)
        try:
            for c in range(3):
                wire[:] = 0
                enc.tx_assemble_host(pk, pl, wire, wl, pad=pad, max_len=L)
                keepb = np.arange(slot)[None, :] < want_tx[1][:, None].astype(np.int64)
                got[f"tx{c}"] = bool(np.array_equal(wl, want_tx[1])) and bool(
                    np.array_equal(wire[keepb], want_tx[0][keepb]))
        finally:
            enc.close()

    def rx():
        enc = fec.New(d, p)
        try:
            for c in range(3):
                nrec, index, out, _ = enc.rx_recover_host(ring, rlens, S, G, pad=pad)
                got[f"rx{c}"] = nrec == k and bool(np.array_equal(index[:k], want_rx[0])) and bool(
                    np.array_equal(out[:k, :S], want_rx[1]))
        finally:
            enc.close()

    def staged():
        enc = fec.New(d, p)
        try:
            for c in range(3):
                b = host_enc.copy()
                enc.encode_host(b, 1350)
                got[f"enc{c}"] = bool(np.array_equal(b[:, :, :1350], want_enc[:, :, :1350]))
        finally:
            enc.close()

    def guard(fn):
        try:
            fn()
        except BaseException as e:
            errs.append((fn.__name__, repr(e)))

    try:
        ths = [threading.Thread(target=guard, args=(f,)) for f in (tx, rx, staged)]
        for t in ths:
            t.start()
        for t in ths:
            t.join(timeout=300)
        assert not any(t.is_alive() for t in ths)
        assert not errs, errs
        assert got == {f"{w}{c}": True for w in ("tx", "rx", "enc") for c in range(3)}, got
    finally:
        for a in bufs:
            fec.host_free(a.reshape(-1).view(np.uint8))
        ref.close()
