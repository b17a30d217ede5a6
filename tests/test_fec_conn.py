"""The C++ host mirror of ugo's FEC object (include/ugo_fec_conn.h) against the
pure-Python restatement of ugo/fec.go (oracle/fec_ref.py, checker only).

TX: markData / calcECC / markFEC exactly as the (commented) sender loop
ugo/conn.go:643-685 drives them, with the 13 reused, never-zeroed group buffers.
RX: Conn.handlePacket's hook (ugo/conn.go:394-396) over a lossy channel with
drops, duplicates, local reordering, junk flags and clock jumps past fecExpire.
Both sides see the same packets and the same injected clock; every step's
(seqid, flag, recovered shards) and len(rx) must match bit for bit.  The
C++ side computes all Reed-Solomon bytes on the GPU.
"""
import os

import numpy as np
import pytest
from hypothesis import HealthCheck, event, given, settings
from hypothesis import strategies as st

import fec_ref
from ugo_amd import fec

D, P, N, RXLIMIT = 10, 3, 13, 128


def test_newfec_geometry_rejected_without_device():
    # newFEC returns nil before constructing an encoder (ugo/fec.go:46-51)
    for args in [(128, 0, 3), (128, 10, 0), (12, 10, 3), (128, -1, 3)]:
        with pytest.raises(fec.ErrInvShardNum):
            fec.FecConn(*args)
        assert fec_ref.FEC.new(*args, clock=lambda: 0) is None


def test_oracle_paws_and_headers():
    f = fec_ref.FEC.new(RXLIMIT, D, P, clock=lambda: 0)
    assert f.paws == (0xFFFFFFFF // 13 - 1) * 13 == 4294967274
    b = bytearray(8)
    f.next = f.paws - 1
    f.markFEC(b)
    assert b[:6] == (f.paws - 1).to_bytes(4, "little") + bytes([0xF2, 0x00]) and f.next == 0
    f.markData(b)
    assert b[:6] == bytes([0, 0, 0, 0, 0xF1, 0]) and f.next == 1


def _tx_stream(tx, groups, rng, full_len):
    """The sender loop of ugo/conn.go:643-685 (markData, copy into fecGroup,
    calcECC at dataShards, markFEC, send ecc[:fecMaxSize])."""
    packets, originals = [], []
    group = [bytearray(fec_ref.maxPacketSize) for _ in range(N)]  # reused, never zeroed (:649-653)
    for _ in range(groups):
        maxsize = 0
        for k in range(D):
            L = fec_ref.maxPacketSize if full_len else int(rng.integers(7, fec_ref.maxPacketSize + 1))
            ori = bytearray(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
            tx.markData(ori)
            group[k][:L] = ori
            maxsize = max(maxsize, L)
            packets.append(bytes(ori))
            originals.append(bytes(ori))
        ecc = tx.calcECC(group, fec_ref.fecHeaderSize, maxsize)
        assert ecc is not None and len(ecc) == P
        for k in range(P):
            tx.markFEC(ecc[k])
            packets.append(bytes(ecc[k][:maxsize]))
    return packets, originals


def _channel(packets, rng, drop, dup, junk, reorder=4):
    out = []
    for pkt in packets:
        if rng.random() < junk:
            j = bytearray(rng.integers(0, 256, int(rng.integers(7, 200)), dtype=np.uint8).tobytes())
            j[4:6] = b"\x34\x12"  # neither typeData nor typeFEC
            out.append(bytes(j))
        if rng.random() < drop:
            continue
        out.append(pkt)
        if rng.random() < dup:
            out.append(pkt)
    for i in range(0, len(out) - reorder, reorder):  # local reordering
        win = out[i:i + reorder]
        rng.shuffle(win)
        out[i:i + reorder] = win
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("full_len,drop,seed,service", [(True, 0.12, 1, False), (False, 0.12, 2, False),
                                                         (False, 0.3, 3, False), (True, 0.12, 1, True),
                                                         (False, 0.3, 3, True)])
def test_fec_object_lockstep_with_reference_restatement(gpu, full_len, drop, seed, service):
    """service: calcECC's Encode and the per-call Reconstruct served by the
    resident workgroup (ugo_fecconn_service) -- the same bytes."""
    rng = np.random.default_rng(seed)
    now = [1_000_000]
    clock = lambda: now[0]  # noqa: E731

    # TX: C++ mirror (GPU parity) vs oracle restatement, byte for byte
    tx_c = fec.FecConn(RXLIMIT, D, P)
    if service:
        tx_c.service()
    tx_o = fec_ref.FEC.new(RXLIMIT, D, P, clock)
    pk_c, orig = _tx_stream(tx_c, 40, np.random.default_rng(seed), full_len)
    pk_o, _ = _tx_stream(tx_o, 40, np.random.default_rng(seed), full_len)
    assert pk_c == pk_o, "TX packets (markData / calcECC / markFEC) differ from the reference restatement"
    assert tx_c.next == tx_o.next

    # RX over a lossy channel
    rx_c = fec.FecConn(RXLIMIT, D, P)
    rx_c.set_clock(clock)
    if service:
        rx_c.service(500)
    rx_o = fec_ref.FEC.new(RXLIMIT, D, P, clock)
    wire = _channel(pk_c, rng, drop=drop, dup=0.05, junk=0.02)
    recovered_total = 0
    for i, pkt in enumerate(wire):
        now[0] += int(rng.integers(0, 40))
        if i == len(wire) // 2:
            now[0] += fec_ref.fecExpire + 1  # expiry sweep (ugo/fec.go:109-121)
        sc, fc, rc = rx_c.input(pkt)
        so, fo, ro = fec_ref.handle(rx_o, pkt)
        assert (sc, fc) == (so, fo)
        assert (rc is None) == (ro is None), f"step {i}: recovered {rc is not None} vs {ro is not None}"
        if rc is not None:
            assert [bytes(x) for x in rc] == [bytes(x) for x in ro], f"step {i}: recovered bytes differ"
            recovered_total += len(rc)
            if full_len:  # consistent codewords: recovery restores the lost payloads
                base = so - so % N
                lost = [k for k in range(D)]
                payloads = {bytes(orig[(base // N) * D + k][6:]) for k in lost}
                for x in rc:
                    assert bytes(x[:1470]) in payloads
        assert rx_c.rx_len() == len(rx_o.rx), f"step {i}: len(rx)"
    assert recovered_total > 0


@pytest.mark.gpu
def test_calc_ecc_mismatch_and_window(gpu):
    f = fec.FecConn(RXLIMIT, D, P)
    with pytest.raises(fec.FecError):
        f.calcECC([bytearray(100) for _ in range(12)], 6, 50)  # len(data) != shardSize: "mismatch"
    rng = np.random.default_rng(5)
    bufs = [bytearray(rng.integers(0, 256, 1476, dtype=np.uint8).tobytes()) for _ in range(N)]
    ref = [bytearray(b) for b in bufs]
    f.calcECC(bufs, 6, 900)
    o = fec_ref.FEC.new(RXLIMIT, D, P, clock=lambda: 0)
    o.calcECC(ref, 6, 900)
    assert bufs == ref  # parity in [6, 900) only; bytes outside the window untouched


@pytest.mark.gpu
def test_paws_wrap_on_device_object(gpu):
    f = fec.FecConn(RXLIMIT, D, P)
    f.next = 4294967274 - 1
    b = bytearray(16)
    f.markFEC(b)
    assert f.next == 0 and b[4:6] == b"\xf2\x00"


@pytest.mark.gpu
@pytest.mark.parametrize("batch,overlap", [(1, False), (4, False), (7, False), (1, True), (4, True), (7, True),
                                           (64, True)])
def test_batched_recovery_is_per_call_recovery_delayed(gpu, batch, overlap):
    """set_batch(n): recoverable lossy groups are staged and recovered n per
    launch, their survivors read by the GPU in the pinned pool buffers decode
    filled (short packets, so the buffers' stale tails matter, and buffers
    are reused while a batch still has to read them).  Every step's
    (seqid, flag) and len(rx) equal the reference restatement's; the
    recovered shards, concatenated over the run and the final flush, equal the
    per-call sequence byte for byte, and what has come back at any step is a
    prefix of it.  overlap: each batch runs while the next one fills and
    comes back one batch later."""
    rng = np.random.default_rng(20 + batch)
    now = [2_000_000]
    clock = lambda: now[0]  # noqa: E731
    tx = fec_ref.FEC.new(RXLIMIT, D, P, clock)
    pk, _ = _tx_stream(tx, 60, np.random.default_rng(batch), False)
    wire = _channel(pk, rng, drop=0.15, dup=0.05, junk=0.02)
    rx_b = fec.FecConn(RXLIMIT, D, P)
    rx_b.set_clock(clock)
    assert rx_b.set_batch(batch, overlap=overlap) is None
    rx_o = fec_ref.FEC.new(RXLIMIT, D, P, clock)
    got, want = [], []
    for i, pkt in enumerate(wire):
        now[0] += int(rng.integers(0, 40))
        if i == len(wire) // 2:
            now[0] += fec_ref.fecExpire + 1
        sb, fb, rb = rx_b.input(pkt)
        so, fo, ro = fec_ref.handle(rx_o, pkt)
        assert (sb, fb) == (so, fo)
        assert rx_b.rx_len() == len(rx_o.rx), f"step {i}: len(rx)"
        assert rx_b.pending() < (2 if overlap else 1) * batch
        got += [bytes(x) for x in rb or []]
        want += [bytes(x) for x in ro or []]
        assert got == want[:len(got)], f"step {i}: recovered shards out of order or different"
    pending = rx_b.pending()
    got += [bytes(x) for x in rx_b.flush() or []]
    assert rx_b.pending() == 0
    assert got == want and len(want) > 0
    if batch > 1 and not overlap:
        assert pending > 0 or len(want) % batch == 0


@pytest.mark.gpu
def test_set_batch_flushes_pending_and_rejects_bad_sizes(gpu):
    rng = np.random.default_rng(31)
    tx = fec_ref.FEC.new(RXLIMIT, D, P, clock=lambda: 0)
    pk, _ = _tx_stream(tx, 6, np.random.default_rng(31), True)
    rx_o = fec_ref.FEC.new(RXLIMIT, D, P, clock=lambda: 0)
    rx_b = fec.FecConn(RXLIMIT, D, P)
    rx_b.set_clock(lambda: 0)
    rx_b.set_batch(64)
    want = []
    for g in range(6):  # drop data shard g % D of every group: 6 lossy groups
        for k, pkt in enumerate(pk[g * N:(g + 1) * N]):
            if k == g % D:
                continue
            _, _, rb = rx_b.input(pkt)
            assert rb is None, "nothing comes back before the batch is full"
            want += [bytes(x) for x in fec_ref.handle(rx_o, pkt)[2] or []]
    assert rx_b.pending() == 6 and len(want) == 6
    with pytest.raises(fec.FecError):
        rx_b.set_batch(-1)
    assert rx_b.pending() == 6, "a refused set_batch consumes nothing"
    got = rx_b.set_batch(0)  # back to per call: the pending groups come back first
    assert [bytes(x) for x in got] == want and rx_b.pending() == 0
    del rng


@pytest.mark.gpu
def test_input_refuses_a_short_output_buffer_before_consuming(gpu):
    """Per-call input needs room for d recovered shards up front: a shorter
    buffer is refused and the packet is not taken into the rx queue."""
    import ctypes

    tx = fec_ref.FEC.new(RXLIMIT, D, P, clock=lambda: 0)
    pk, _ = _tx_stream(tx, 1, np.random.default_rng(5), True)
    rx = fec.FecConn(RXLIMIT, D, P)
    rx.set_clock(lambda: 0)
    w = (ctypes.c_uint8 * len(pk[0])).from_buffer_copy(pk[0])
    small = (ctypes.c_uint8 * ((D - 1) * fec.UGO_FEC_MAX_PACKET))()
    nrec, rlen = ctypes.c_int(), ctypes.c_size_t()
    st = rx._lib.ugo_fecconn_input(rx._h, ctypes.addressof(w), len(pk[0]), None, None, ctypes.addressof(small),
                                   len(small), ctypes.byref(nrec), ctypes.byref(rlen))
    assert st == fec.ErrInvalidArg.code and rx.rx_len() == 0
    rx.input(pk[0])  # the binding's own buffer holds d shards
    assert rx.rx_len() == 1
    # overlapped batches of 4: input must hold two batches (the pinned-exhaustion
    # fallback returns both); one batch's worth is refused, nothing consumed
    rx.set_batch(4, overlap=True)
    one_batch = (ctypes.c_uint8 * (4 * D * fec.UGO_FEC_MAX_PACKET))()
    w1 = (ctypes.c_uint8 * len(pk[1])).from_buffer_copy(pk[1])
    st = rx._lib.ugo_fecconn_input(rx._h, ctypes.addressof(w1), len(pk[1]), None, None, ctypes.addressof(one_batch),
                                   len(one_batch), ctypes.byref(nrec), ctypes.byref(rlen))
    assert st == fec.ErrInvalidArg.code and rx.rx_len() == 1
    rx.input(pk[1])
    assert rx.rx_len() == 2


def _tx_stream_any(tx, d, p, groups, rng, max_len):
    """_tx_stream for any (d, p): the sender loop with reused group buffers."""
    n = d + p
    packets = []
    group = [bytearray(fec_ref.maxPacketSize) for _ in range(n)]
    for _ in range(groups):
        maxsize = 0
        for k in range(d):
            L = int(rng.integers(7, max_len + 1))
            ori = bytearray(rng.integers(0, 256, L, dtype=np.uint8).tobytes())
            tx.markData(ori)
            group[k][:L] = ori
            maxsize = max(maxsize, L)
            packets.append(bytes(ori))
        ecc = tx.calcECC(group, fec_ref.fecHeaderSize, maxsize)
        for k in range(p):
            tx.markFEC(ecc[k])
            packets.append(bytes(ecc[k][:maxsize]))
    return packets


@pytest.mark.gpu
@settings(max_examples=int(os.environ.get("UGO_HYP_EXAMPLES_CONN", "40")), deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(d=st.integers(1, 12), p=st.integers(1, 5), extra=st.integers(0, 60), groups=st.integers(1, 30),
       max_len=st.integers(7, fec_ref.maxPacketSize), drop=st.floats(0, 0.6), dup=st.floats(0, 0.3),
       junk=st.floats(0, 0.1), reorder=st.integers(1, 40), batch=st.sampled_from([0, 0, 1, 3, 16, -1, -3, -16]),
       seed=st.integers(0, 2**31 - 1))
def test_fec_object_random_channels(gpu, d, p, extra, groups, max_len, drop, dup, junk, reorder, batch, seed):
    """Random codes and rxlimits, packet sizes, channels (loss, duplicates,
    junk flags, reordering windows up to 40 packets, clock jumps past
    fecExpire) and, with batch > 0, batched recovery: every step's
    (seqid, flag) and len(rx) match the restated ugo/fec.go, and the recovered
    shards match -- per call, or (batched) as the same sequence delayed to the
    flushes (batch < 0: overlapped batches of -batch groups)."""
    n = d + p
    rxlimit = n + extra
    rng = np.random.default_rng(seed)
    now = [5_000_000]
    clock = lambda: now[0]  # noqa: E731
    tx = fec_ref.FEC.new(rxlimit, d, p, clock)
    pk = _tx_stream_any(tx, d, p, groups, rng, max_len)
    wire = _channel(pk, rng, drop=drop, dup=dup, junk=junk, reorder=reorder)
    rx_c = fec.FecConn(rxlimit, d, p)
    rx_c.set_clock(clock)
    if batch:
        rx_c.set_batch(abs(batch), overlap=batch < 0)
    rx_o = fec_ref.FEC.new(rxlimit, d, p, clock)
    got, want = [], []
    for i, pkt in enumerate(wire):
        now[0] += int(rng.integers(0, 50))
        if rng.random() < 0.01:
            now[0] += fec_ref.fecExpire + 1
        sc, fc, rc = rx_c.input(pkt)
        so, fo, ro = fec_ref.handle(rx_o, pkt)
        assert (sc, fc) == (so, fo), i
        assert rx_c.rx_len() == len(rx_o.rx), i
        if rc is not None:
            got += [bytes(x) for x in rc]
        if ro is not None:
            want += [bytes(x) for x in ro]
        if not batch:
            assert (rc is None) == (ro is None), i
    if batch:
        rc = rx_c.flush()
        if rc is not None:
            got += [bytes(x) for x in rc]
    assert got == want
    event(f"recovered shards: {'none' if not want else ('1-9' if len(want) < 10 else '10+')}")


@pytest.mark.gpu
@settings(max_examples=int(os.environ.get("UGO_HYP_EXAMPLES_CONN", "40")), deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(d=st.integers(1, 12), p=st.integers(1, 5), offset=st.integers(0, 40), width=st.integers(0, 1476),
       buflen=st.integers(0, 200), seed=st.integers(0, 2**31 - 1))
def test_calc_ecc_random_windows(gpu, d, p, offset, width, buflen, seed):
    """calcECC(data, offset, maxlen) on random codes and windows, buffers
    longer than the window: parity bytes in [offset, maxlen) and every byte
    outside it equal the restated ugo/fec.go (an empty window: Encode fails,
    calcECC returns nil and writes nothing)."""
    n = d + p
    maxlen = offset + width
    rng = np.random.default_rng(seed)
    bufs = [bytearray(rng.integers(0, 256, maxlen + buflen, dtype=np.uint8).tobytes()) for _ in range(n)]
    ref = [bytearray(b) for b in bufs]
    f = fec.FecConn(n + 4, d, p)
    o = fec_ref.FEC.new(n + 4, d, p, clock=lambda: 0)
    want = o.calcECC(ref, offset, maxlen)
    if want is None:
        with pytest.raises(fec.FecError):
            f.calcECC(bufs, offset, maxlen)
    else:
        f.calcECC(bufs, offset, maxlen)
    assert bufs == ref


@pytest.mark.gpu
def test_set_batch_allocation_failure_falls_back_to_per_call(gpu, monkeypatch):
    """a set_batch whose pinned batch cannot be allocated (fault
    injected: ugo_fec_set_host_alloc_limit) fails with ErrHip and leaves the object
    in per-call mode -- it never keeps pointing at a freed batch.  Before and
    after, input recovers exactly what the reference restatement recovers
    (pending groups of the old batch come back first)."""
    rng = np.random.default_rng(41)
    tx = fec_ref.FEC.new(RXLIMIT, D, P, clock=lambda: 0)
    pk, _ = _tx_stream(tx, 12, np.random.default_rng(41), False)
    rx_o = fec_ref.FEC.new(RXLIMIT, D, P, clock=lambda: 0)
    rx_b = fec.FecConn(RXLIMIT, D, P)
    rx_b.set_clock(lambda: 0)
    rx_b.set_batch(4)
    got, want = [], []

    def feed(groups):
        for g in groups:
            for k, pkt in enumerate(pk[g * N:(g + 1) * N]):
                if k == g % D:
                    continue
                _, _, rb = rx_b.input(pkt)
                got.extend(bytes(x) for x in rb or [])
                want.extend(bytes(x) for x in fec_ref.handle(rx_o, pkt)[2] or [])

    feed(range(0, 6))  # one full batch of 4 came back, 2 pending
    assert rx_b.pending() == 2
    import ctypes
    lib = fec._bind_conn(fec.load_library())
    lib.ugo_fec_set_host_alloc_limit.argtypes = [ctypes.c_size_t]
    lib.ugo_fec_set_host_alloc_limit(4096)
    try:
        nrec, rlen = ctypes.c_int(), ctypes.c_size_t()
        st = lib.ugo_fecconn_set_batch_ex(rx_b._h, 8, 0, ctypes.addressof(rx_b._out), len(rx_b._out),
                                          ctypes.byref(nrec), ctypes.byref(rlen))
    finally:
        lib.ugo_fec_set_host_alloc_limit(0)
    assert st == fec.ErrHip.code
    got.extend(bytes(x) for x in rx_b._recovered(nrec, rlen) or [])  # the 2 pending groups, flushed first
    assert rx_b.pending() == 0
    n_before = len(got)
    feed(range(6, 12))  # per-call mode now: every lossy group comes back at once
    assert rx_b.pending() == 0
    assert len(got) == n_before + 6
    assert got == want and len(want) == 12
    del rng
