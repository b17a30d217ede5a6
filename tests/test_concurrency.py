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
