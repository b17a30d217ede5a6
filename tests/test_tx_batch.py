"""TX group assembly (SURVEY §8f rows 2 + 3): header marking + calcECC over the
[6, maxsize) window + RC4 encryption of whole groups on the GPU
(ugo_fec_tx_assemble), bit-exact against the restated sender loop
(oracle/fec_ref.tx_group: ugo/conn.go:643-685 + ugo/conn.go:634) run with the
same seqids; then TX -> lossy channel -> RX assembly -> Reconstruct round trip.
"""
import os

import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import fec_ref
from ugo_amd import fec

KEY = b"1234567890123456"  # ugo/listener.go:92, ugo/dial.go:132


def _paws(n):
    return (0xFFFFFFFF // n - 1) * n


def _batch(d, G, seed, max_len, full_frac=0.3):
    rng = np.random.default_rng(seed)
    lens = rng.integers(7, max_len + 1, G * d)
    lens[rng.random(G * d) < full_frac] = max_len
    lens[::7] = 6  # header-only packets
    pk = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in lens]
    return pk, lens


def _run_gpu(enc, pk, lens, slot, first_seq, key, max_len, status=None):
    d, n = enc.DataShards, enc.Shards
    G = len(pk) // d
    host = np.zeros((G * d, slot), np.uint8)
    for i, b in enumerate(pk):
        host[i, :min(len(b), slot)] = np.frombuffer(b[:slot], np.uint8)
    dp = torch.from_numpy(host).cuda()
    dl = torch.from_numpy(lens.astype(np.int16)).cuda()
    wire = torch.full((G * n, slot), 0xAB, dtype=torch.uint8, device="cuda")
    wl = torch.zeros(G * n, dtype=torch.int16, device="cuda")
    pad = None
    if key is not None:
        pad = torch.frombuffer(bytearray(fec.rc4_keystream(key, slot)), dtype=torch.uint8).cuda()
    enc.tx_assemble(dp, dl, wire, wl, first_seq=first_seq, pad=pad, max_len=max_len, status=status)
    torch.cuda.synchronize()
    return wire.cpu().numpy(), wl.cpu().numpy().astype(np.int64) & 0xFFFF


def _oracle(d, p, pk, first_seq, key):
    tx = fec_ref.FEC.new(128, d, p, clock=lambda: 0)
    tx.next = first_seq
    out = []
    for g in range(len(pk) // d):
        out += fec_ref.tx_group(tx, pk[g * d:(g + 1) * d], key)
    return out, tx.next


def test_oracle_tx_group_matches_reused_buffer_loop_on_full_packets():
    """With full-length packets the stale-tail difference vanishes: tx_group
    (fresh buffers) equals the literal reused-buffer loop of ugo/conn.go:643-685,
    and decrypting + the RX restatement gets every group back without loss."""
    import rc4_ref
    d, p, n = 10, 3, 13
    rng = np.random.default_rng(1)
    pk = [bytes(rng.integers(0, 256, 1476, dtype=np.uint8).tobytes()) for _ in range(4 * d)]
    a, b = fec_ref.FEC.new(128, d, p, clock=lambda: 0), fec_ref.FEC.new(128, d, p, clock=lambda: 0)
    fresh = []
    for g in range(4):
        fresh += fec_ref.tx_group(a, pk[g * d:(g + 1) * d], KEY)
    bufs = [bytearray(fec_ref.maxPacketSize) for _ in range(n)]
    loop = []
    for g in range(4):
        for k in range(d):
            ori = bytearray(pk[g * d + k])
            b.markData(ori)
            bufs[k][:] = ori
            loop.append(rc4_ref.xor_stream(KEY, bytes(ori)))
        ecc = b.calcECC(bufs, 6, 1476)
        for k in range(p):
            b.markFEC(ecc[k])
            loop.append(rc4_ref.xor_stream(KEY, bytes(ecc[k])))
    assert fresh == loop and a.next == b.next == 4 * n


@pytest.mark.gpu
@pytest.mark.parametrize("d,p,max_len,G,key,wrap", [
    (10, 3, 1476, 96, KEY, False),   # headline geometry, compile-time network
    (10, 3, 1476, 40, None, True),   # seqids wrap at paws mid-batch (markFEC)
    (10, 3, 500, 64, KEY, False),    # < 64 chunks per packet: per-lane lengths (a wave spans > 2 groups)
    (5, 3, 1476, 40, KEY, False),    # descriptor kernel
    (12, 4, 700, 24, KEY, False),
    (32, 8, 9006, 6, KEY, False),    # jumbo network
])
def test_tx_assemble_vs_sender_loop(gpu, d, p, max_len, G, key, wrap):
    n = d + p
    enc = fec.New(d, p)
    pk, lens = _batch(d, G, 100 + d, max_len)
    first_seq = _paws(n) - 13 * n if wrap else 26 * n
    slot = (max_len + 15) // 16 * 16
    wire, wl = _run_gpu(enc, pk, lens, slot, first_seq, key, max_len)
    ref, nxt = _oracle(d, p, pk, first_seq, key)
    assert len(ref) == G * n
    for i, w in enumerate(ref):
        assert wl[i] == len(w), f"packet {i}: length {wl[i]} vs {len(w)}"
        assert wire[i, :len(w)].tobytes() == w, f"packet {i} (group {i // n}, row {i % n}) differs"
    if wrap:
        assert nxt < first_seq  # the batch crossed paws, like FEC.next does


@pytest.mark.gpu
@pytest.mark.parametrize("d,p,max_len,G,key,pinned,route", [
    (10, 3, 1476, 97, KEY, True, "copy"),     # headline geometry: >= 4 chunks over the 3 streams
    (10, 3, 1476, 97, KEY, True, "mapped"),   # the kernel writes the pinned wire buffer itself
    (10, 3, 1476, 5, None, False, "mapped"),  # pageable buffers (no mapping: the copy route), one group per chunk
    (5, 3, 700, 33, KEY, True, "copy"),       # descriptor kernel
    (5, 3, 700, 33, KEY, True, "mapped"),
])
def test_tx_assemble_host_vs_sender_loop(gpu, d, p, max_len, G, key, pinned, route):
    """ugo_fec_tx_assemble_host (host memory in and out, chunks pipelined over
    three streams; wire packets by D2H copy or written through the pinned
    buffer's mapping) against the restated sender loop, statuses included."""
    n = d + p
    enc = fec.New(d, p)
    enc.set_tx_host_route(route)
    pk, lens = _batch(d, G, 300 + d + G, max_len)
    slot = (max_len + 15) // 16 * 16
    first_seq = 13 * n

    def buf(shape, dtype):
        if not pinned:
            return np.zeros(shape, dtype)
        a = fec.host_alloc(int(np.prod(shape)) * np.dtype(dtype).itemsize).view(dtype).reshape(shape)
        a[:] = 0
        return a

    host = buf((G * d, slot), np.uint8)
    for i, b in enumerate(pk):
        host[i, :len(b)] = np.frombuffer(b, np.uint8)
    hl = buf((G * d,), np.uint16)
    hl[:] = lens
    wire, wl, st = buf((G * n, slot), np.uint8), buf((G * n,), np.uint16), buf((G,), np.int8)
    wire[:] = 0xAB
    st[:] = -1
    pad = None if key is None else fec.rc4_keystream(key, slot)
    enc.tx_assemble_host(host, hl, wire, wl, first_seq=first_seq, pad=pad, max_len=max_len, status=st)
    ref, _ = _oracle(d, p, pk, first_seq, key)
    for i, w in enumerate(ref):
        assert wl[i] == len(w), f"packet {i}: length {wl[i]} vs {len(w)}"
        assert wire[i, :len(w)].tobytes() == w, f"packet {i} (group {i // n}, row {i % n}) differs"
    nodata = [all(int(L) == 6 for L in lens[g * d:(g + 1) * d]) for g in range(G)]
    assert list(st) == [fec.ErrShardNoData.code if x else 0 for x in nodata]
    if pinned:
        for a in (host, hl, wire, wl, st):
            fec.host_free(a.reshape(-1).view(np.uint8))


@pytest.mark.gpu
@pytest.mark.parametrize("route,copy_queue,service", [("copy", False, False), ("mapped", False, False),
                                                     ("copy", True, False), ("copy", True, True)])
def test_tx_assemble_host_many_chunks_matches_device_path(gpu, route, copy_queue, service):
    """A batch past tx_assemble_host's chunk cap (32 chunks per call; the
    chunks grow with the batch): 3,400 (32,8) groups of up to 9,006-B packets
    in pinned memory, against the device-resident tx_assemble (itself checked
    against the sender loop above) -- every wire packet within its length,
    the wire lengths and the statuses, header-only and bad groups included.
    Two calls on the context, each checked; copy_queue: the first two with the
    low-priority copy stream (ugo_fec_set_host_copy_queue, the default), a
    third after switching it off again.  service: another context's per-call
    service block stays resident (polling, 2-s idle window) through the calls,
    as in a process where connections use the drop-in route beside the batch
    route."""
    d, p, max_len, G = 32, 8, 9006, 3400
    n, slot = d + p, (max_len + 15) // 16 * 16
    enc = fec.New(d, p)
    enc.set_tx_host_route(route)
    enc.set_host_copy_queue(copy_queue)
    gen = torch.Generator(device="cuda").manual_seed(77)
    dp = torch.randint(0, 256, (G * d, slot), dtype=torch.uint8, device="cuda", generator=gen)
    ln = torch.randint(6, max_len + 1, (G * d,), dtype=torch.int32, device="cuda", generator=gen)
    ln[7 * d:8 * d] = 6         # a header-only group: no parity
    ln[11 * d + 3] = 5          # a bad group
    ln = ln.to(torch.int16)
    pad = fec.rc4_keystream(KEY, slot)
    dw = torch.empty((G * n, slot), dtype=torch.uint8, device="cuda")
    dwl = torch.empty(G * n, dtype=torch.int16, device="cuda")
    dst = torch.empty(G, dtype=torch.int8, device="cuda")
    enc.tx_assemble(dp, ln, dw, dwl, pad=torch.frombuffer(bytearray(pad), dtype=torch.uint8).cuda(),
                    max_len=max_len, status=dst)
    bufs = []

    def pinned(nbytes):
        a = fec.host_alloc(nbytes)
        bufs.append(a)
        return a

    svc = None
    try:
        if service:
            svc = fec.New(10, 3)  # a (10,3) connection: the service serves codes up to d = 16
            svc.service_start(idle_us=2_000_000)
            one = pinned(13 * 16).reshape(1, 13, 16)
            one[:] = 3
            svc.encode_host(one, 16)  # served: the block is now resident
        hp = pinned(G * d * slot).reshape(G * d, slot)
        hl = pinned(G * d * 2).view(np.uint16)
        hw = pinned(G * n * slot).reshape(G * n, slot)
        hwl = pinned(G * n * 2).view(np.uint16)
        hst = pinned(G).view(np.int8)
        torch.from_numpy(hp).copy_(dp)
        hl[:] = ln.cpu().numpy().view(np.uint16)
        want_l = dwl.cpu().numpy().view(np.uint16)
        keep = torch.arange(slot, device="cuda")[None, :] < dwl.to(torch.int32).view(-1, 1)
        for call in range(3 if copy_queue else 2):
            if call == 2:
                enc.set_host_copy_queue(False)  # the stream is replaced between calls
            hst[:] = -1
            hwl[:] = 0
            hw[:, :64] = 0xAB
            enc.tx_assemble_host(hp, hl, hw, hwl, pad=pad, max_len=max_len, status=hst)
            assert np.array_equal(hwl, want_l), f"call {call}"
            assert np.array_equal(hst, dst.cpu().numpy()), f"call {call}"
            got = torch.from_numpy(hw).cuda()
            assert torch.equal(got[keep], dw[keep]), f"call {call}"
            del got
    finally:
        if svc is not None:
            svc.service_stop()
            svc.close()
        for a in bufs:
            fec.host_free(a)


@pytest.mark.gpu
def test_tx_assemble_bad_length_group_and_arguments(gpu):
    d, p, n = 10, 3, 13
    enc = fec.New(d, p)
    pk, lens = _batch(d, 8, 3, 1476)
    lens = lens.copy()
    lens[2 * d + 4] = 5  # too short for the FEC header: group 2 rejected
    lens[5 * d + 9] = 1477  # above max_len: group 5 rejected
    st = torch.full((8,), -1, dtype=torch.int8, device="cuda")
    wire, wl = _run_gpu(enc, pk, lens, 1488, 0, KEY, 1476, status=st)
    s = st.cpu().numpy()
    assert list(s) == [0, 0, fec.ErrShardSize.code, 0, 0, fec.ErrShardSize.code, 0, 0]
    assert not wl[2 * n:3 * n].any() and not wl[5 * n:6 * n].any()
    # the groups before it are unaffected: same bytes as the oracle on them alone
    ref, _ = _oracle(d, p, pk[:2 * d], 0, KEY)
    for i, w in enumerate(ref):
        assert wire[i, :len(w)].tobytes() == w
    with pytest.raises(fec.ErrInvalidArg):  # first_seq not at a group boundary
        _run_gpu(enc, pk, lens, 1488, 7, KEY, 1476)
    with pytest.raises(fec.ErrInvalidArg):  # slot smaller than max_len
        _run_gpu(enc, pk, lens, 1472, 0, KEY, 1476)


@pytest.mark.gpu
def test_tx_lossy_rx_reconstruct_round_trip(gpu):
    """TX batch -> drop <= p packets per group -> RX batch -> Reconstruct: every
    data payload comes back (zero-padded to the row) bit for bit."""
    d, p, n, S, pitch, slot = 10, 3, 13, 1470, 1472, 1488
    G = 512
    enc = fec.New(d, p)
    pk, lens = _batch(d, G, 9, 1476)
    wire, wl = _run_gpu(enc, pk, lens, slot, 0, KEY, 1476)
    rng = np.random.default_rng(10)
    keep = []
    for g in range(G):
        lost = set(rng.choice(n, int(rng.integers(0, p + 1)), replace=False).tolist())
        keep += [g * n + r for r in range(n) if r not in lost]
    keep = np.array(keep)
    rng.shuffle(keep)
    rx = torch.from_numpy(np.ascontiguousarray(wire[keep])).cuda()
    rl = torch.from_numpy(wl[keep].astype(np.int16)).cuda()
    pad = torch.frombuffer(bytearray(fec.rc4_keystream(KEY, slot)), dtype=torch.uint8).cuda()
    sh = torch.zeros((n, G, pitch), dtype=torch.uint8, device="cuda")
    present = torch.zeros(G, dtype=torch.int64, device="cuda")
    enc.rx_assemble(rx, rl, sh, present, shard_size=S, pad=pad)
    enc.reconstruct_batch(sh, present, shard_size=S, data_only=True, shard_major=True)
    got = sh.cpu().numpy()
    for g in range(G):
        for k in range(d):
            b = pk[g * d + k]
            want = np.zeros(S, np.uint8)
            want[:len(b) - 6] = np.frombuffer(b[6:], np.uint8)
            assert np.array_equal(got[k, g, :S], want), f"group {g} row {k}"


@pytest.mark.gpu
def test_tx_rx_round_trip_full_size(gpu):
    """BASELINE size (65,536 groups of (10+3), 1476-B packets), all on the
    device: TX assemble -> lose 0..3 packets per group -> shuffle -> RX
    assemble -> data-only Reconstruct.  Size-independent property: every data
    payload comes back bit for bit (zero-padded past its length), and every
    group is recoverable."""
    d, p, n, S, pitch, slot, G = 10, 3, 13, 1470, 1472, 1488, 65536
    dev = "cuda"
    gen = torch.Generator(device=dev).manual_seed(21)
    enc = fec.New(d, p)
    pk = torch.randint(0, 256, (G * d, slot), dtype=torch.uint8, device=dev, generator=gen)
    lens = torch.randint(7, 1477, (G * d,), dtype=torch.int16, device=dev, generator=gen)
    lens[torch.rand(G * d, device=dev, generator=gen) < 0.5] = 1476
    wire = torch.empty((G * n, slot), dtype=torch.uint8, device=dev)
    wl = torch.empty(G * n, dtype=torch.int16, device=dev)
    pad = torch.frombuffer(bytearray(fec.rc4_keystream(KEY, slot)), dtype=torch.uint8).to(dev)
    st = torch.full((G,), -1, dtype=torch.int8, device=dev)
    enc.tx_assemble(pk, lens, wire, wl, pad=pad, status=st)
    assert bool((st == 0).all())
    # lose e ~ U[0, 3] distinct packets per group: rank random keys within each group
    e = torch.randint(0, p + 1, (G, 1), device=dev, generator=gen)
    rank = torch.rand((G, n), device=dev, generator=gen).argsort(dim=1).argsort(dim=1)
    keep = (rank >= e).reshape(-1).nonzero().squeeze(1)
    keep = keep[torch.randperm(keep.numel(), device=dev, generator=gen)]
    rx, rl = wire[keep].contiguous(), wl[keep].contiguous()
    del wire
    sh = torch.zeros((n, G, pitch), dtype=torch.uint8, device=dev)
    present = torch.zeros(G, dtype=torch.int64, device=dev)
    stats = torch.zeros(5, dtype=torch.int32, device=dev)
    enc.rx_assemble(rx, rl, sh, present, shard_size=S, pad=pad, stats=stats)
    assert stats.tolist() == [keep.numel(), 0, 0, 0, 0]
    status = torch.full((G,), -1, dtype=torch.int8, device=dev)
    enc.reconstruct_batch(sh, present, shard_size=S, data_only=True, status=status, shard_major=True)
    assert bool((status == 0).all())
    # expected rows: payload bytes [6, len) of each data packet, zero past it
    col = torch.arange(S, device=dev)
    for k in range(d):  # one data row at a time keeps the temporaries small
        pkt = pk.view(G, d, slot)[:, k, 6:6 + S]
        L = (lens.view(G, d)[:, k].to(torch.int64) - 6).unsqueeze(1)
        want = torch.where(col.unsqueeze(0) < L, pkt, torch.zeros_like(pkt))
        assert torch.equal(sh[k, :, :S], want), f"data row {k}"


@pytest.mark.gpu
@settings(max_examples=int(os.environ.get("UGO_HYP_EXAMPLES_TX", "60")), deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(d=st.integers(1, 32), p=st.integers(1, 8), max_len=st.integers(6, 1600), G=st.integers(1, 24),
       group0=st.integers(0, 40), full=st.floats(0, 1), encrypt=st.booleans(), seed=st.integers(0, 2**31 - 1))
def test_tx_assemble_random_batches(gpu, d, p, max_len, G, group0, full, encrypt, seed):
    """Random codes (d <= 32, the TX kernels' range), packet-length limits,
    length mixes and first seqids: every wire packet and length equals the
    restated sender loop's."""
    n = d + p
    enc = fec.New(d, p)
    rng = np.random.default_rng(seed)
    lens = rng.integers(6, max_len + 1, G * d)
    lens[rng.random(G * d) < full] = max_len
    pk = [rng.integers(0, 256, int(L), dtype=np.uint8).tobytes() for L in lens]
    first_seq = group0 * n
    slot = (max_len + 15) // 16 * 16
    key = KEY if encrypt else None
    st_ = torch.full((G,), -1, dtype=torch.int8, device="cuda")
    wire, wl = _run_gpu(enc, pk, lens, slot, first_seq, key, max_len, status=st_)
    tx = fec_ref.FEC.new(128, d, p, clock=lambda: 0)
    for g in range(G):
        # a group whose packets are all header-only gets no parity (calcECC: empty
        # window); the reference's next then moves by d only, the batch keeps n
        # seqids per group (include/ugo_fec.h)
        tx.next = first_seq + g * n
        out = fec_ref.tx_group(tx, pk[g * d:(g + 1) * d], key)
        nowin = all(len(x) == 6 for x in pk[g * d:(g + 1) * d])
        assert len(out) == (d if nowin else n)
        assert int(st_[g]) == (fec.ErrShardNoData.code if nowin else 0)
        for k, w in enumerate(out):
            i = g * n + k
            assert wl[i] == len(w), (i, wl[i], len(w))
            assert wire[i, :len(w)].tobytes() == w, (i, g, k)
        for k in range(len(out), n):
            assert wl[g * n + k] == 0
