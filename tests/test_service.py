"""Per-call latency service (ugo_fec_service_start): small pinned host batches
served by the resident k_service workgroup give the same bytes and statuses as
the launch path and the oracle, across idle exits and relaunches, stops, and
batches the service does not take.  Oracle = checker only.
"""
import time

import numpy as np
import pytest

import rs_ref
from ugo_amd import fec

pytestmark = pytest.mark.gpu


def _pinned(G, n, pitch, rng):
    buf = fec.host_alloc(G * n * pitch).reshape(G, n, pitch)
    buf[:] = rng.integers(0, 256, (G, n, pitch), dtype=np.uint8)
    return buf


def _masks(G, n, p, rng):
    m = np.zeros(G, np.uint64)
    for g in range(G):
        v = (1 << n) - 1
        for r in rng.choice(n, size=int(rng.integers(0, p + 2)), replace=False):  # includes too-few-shards
            v &= ~(1 << int(r))
        m[g] = v
    return m


def _timed_launches(enc, fn):
    enc.timing_begin(64)
    fn()
    times, untimed = enc.timing_end()
    return len(times) + untimed


@pytest.mark.parametrize("d,p,S,G", [(10, 3, 1470, 1), (10, 3, 1476, 1), (10, 3, 1350, 16), (4, 2, 17, 5),
                                     (12, 4, 1000, 3), (16, 4, 64, 2), (10, 3, 1, 7), (1, 1, 1476, 2)])
def test_service_encode_and_reconstruct_vs_oracle(gpu, d, p, S, G):
    n = d + p
    pitch = (S + 15) // 16 * 16
    rng = np.random.default_rng(S * 7 + G + d)
    enc = fec.New(d, p)
    enc.service_start()
    buf = _pinned(G, n, pitch, rng)
    try:
        want = buf.copy()
        rs_ref.c_encode(d, p, want, S=S)
        assert _timed_launches(enc, lambda: enc.encode_host(buf, S)) == 0  # served by the resident block
        assert np.array_equal(buf[:, :, :S], want[:, :, :S])
        assert np.array_equal(buf[:, :, S:], want[:, :, S:]), "padding written"
        masks = _masks(G, n, p, rng)
        for data_only in (False, True):
            inp = want.copy()
            for g in range(G):
                for r in range(n):
                    if not (int(masks[g]) >> r) & 1:
                        inp[g, r, :S] = 0xEE
            exp = inp.copy()
            rc_want, st_want = rs_ref.c_reconstruct(d, p, exp, masks, S=S, data_only=data_only)
            buf[:] = inp
            st = np.full(G, -1, np.int8)
            rc = None

            def run():
                nonlocal rc
                rc = enc.reconstruct_host(buf, masks, S, data_only, st)
            if n <= 16:
                assert _timed_launches(enc, run) == 0
            else:
                run()
            assert np.array_equal(st, st_want)
            assert rc == (next((int(v) for v in st_want if v), 0))
            assert np.array_equal(buf, exp)
    finally:
        enc.service_stop()
        fec.host_free(buf.reshape(-1))
        enc.close()


def test_service_idle_exit_relaunch_and_stop(gpu):
    """A short idle window: the block leaves between calls and the next call
    relaunches it; many back-to-back calls keep one block; after stop, calls
    take the launch path; batches over 16 groups never use the service."""
    d, p, S = 10, 3, 1470
    n, pitch = d + p, 1472
    rng = np.random.default_rng(5)
    enc = fec.New(d, p)
    enc.service_start(idle_us=200)
    bufs = [_pinned(1, n, pitch, rng), _pinned(40, n, pitch, rng)]
    try:
        for i in range(300):
            b = bufs[0]
            b[:] = rng.integers(0, 256, b.shape, dtype=np.uint8)
            want = b.copy()
            rs_ref.c_encode(d, p, want, S=S)
            enc.encode_host(b, S)
            assert np.array_equal(b[:, :, :S], want[:, :, :S]), i
            if i % 50 == 7:
                time.sleep(0.003)  # > idle: the block has left; the next call relaunches it
        big = bufs[1]
        want = big.copy()
        rs_ref.c_encode(d, p, want, S=S)
        assert _timed_launches(enc, lambda: enc.encode_host(big, S)) > 0  # 40 groups: launch path
        assert np.array_equal(big[:, :, :S], want[:, :, :S])
        enc.service_stop()
        b = bufs[0]
        want = b.copy()
        rs_ref.c_encode(d, p, want, S=S)
        assert _timed_launches(enc, lambda: enc.encode_host(b, S)) > 0  # stopped: launch path
        assert np.array_equal(b[:, :, :S], want[:, :, :S])
        enc.service_start()
        enc.encode_host(b, S)  # restarted
        assert np.array_equal(b[:, :, :S], want[:, :, :S])
    finally:
        enc.service_stop()
        for b in bufs:
            fec.host_free(b.reshape(-1))
        enc.close()


def test_service_serves_the_cgo_shim_sequence(gpu):
    """The cgo shim's own call sequence (replayed by
    test_cgo_shim_replay.GoShim: one pinned stage at the 16-B pitch, groups = 1)
    with the service on: every Encode / Reconstruct / ReconstructData is served
    without a launch, and the shards equal the oracle's and a launch-path
    shim's call for call."""
    from test_cgo_shim_replay import GoShim
    d, p = 10, 3
    rng = np.random.default_rng(9)
    a, b = GoShim(d, p), GoShim(d, p)
    a.ServiceStart(0)
    try:
        for i in range(60):
            S = (1470, 1476)[i % 2]
            data = [bytearray(rng.integers(0, 256, S, dtype=np.uint8).tobytes()) for _ in range(d)]
            sa = [bytearray(x) for x in data] + [bytearray(S) for _ in range(p)]
            sb = [bytearray(x) for x in data] + [bytearray(S) for _ in range(p)]
            a.timing_begin()
            a.Encode(sa)
            lost = rng.choice(d + p, size=int(rng.integers(1, p + 1)), replace=False)
            ra = [None if r in lost else bytearray(x) for r, x in enumerate(sa)]
            (a.ReconstructData if i % 3 == 1 else a.Reconstruct)(ra)
            assert len(a.timing_end()) == 0, "a per-group call launched a kernel"
            b.Encode(sb)
            rb = [None if r in lost else bytearray(x) for r, x in enumerate(sb)]
            (b.ReconstructData if i % 3 == 1 else b.Reconstruct)(rb)
            assert sa == sb and ra == rb
            g = np.zeros((1, d + p, S), np.uint8)
            for k in range(d):
                g[0, k] = np.frombuffer(bytes(data[k]), np.uint8)
            rs_ref.c_encode(d, p, g)
            assert [bytes(x) for x in sa] == [bytes(g[0, k]) for k in range(d + p)]
            for r in range(d):
                assert ra[r] == sa[r]
    finally:
        assert a.lib.ugo_fec_service_stop(a.ctx) == 0
        a.close()
        b.close()


def test_service_two_contexts_from_two_threads(gpu):
    """Two contexts (two connections), each with its own resident service
    block, driven concurrently from two host threads: every call's parity is
    the oracle's."""
    import threading
    d, p, S = 10, 3, 1470
    n, pitch = d + p, 1472
    errors = []

    def worker(seed):
        try:
            rng = np.random.default_rng(seed)
            enc = fec.New(d, p)
            enc.service_start(300)
            b = _pinned(2, n, pitch, rng)
            try:
                for i in range(150):
                    b[:] = rng.integers(0, 256, b.shape, dtype=np.uint8)
                    want = b.copy()
                    rs_ref.c_encode(d, p, want, S=S)
                    enc.encode_host(b, S)
                    if not np.array_equal(b[:, :, :S], want[:, :, :S]):
                        errors.append((seed, i))
                        return
            finally:
                enc.service_stop()
                fec.host_free(b.reshape(-1))
                enc.close()
        except Exception as ex:  # pragma: no cover - reported below
            errors.append((seed, repr(ex)))

    ts = [threading.Thread(target=worker, args=(s,)) for s in (11, 12)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=60)
    assert not any(t.is_alive() for t in ts)
    assert not errors, errors


@pytest.mark.parametrize("d,p,pinned", [(5, 5, True), (20, 4, True), (10, 3, False)])
def test_service_declines_what_it_does_not_serve(gpu, d, p, pinned):
    """p > 4, d > 16 (and d + p > 16: no host-built table to reconstruct
    from), or a pageable batch: with the service on, the calls take the launch
    path and return the oracle's bytes."""
    n, S = d + p, 700
    pitch = 704
    rng = np.random.default_rng(d * 10 + p)
    enc = fec.New(d, p)
    enc.service_start()
    buf = _pinned(3, n, pitch, rng) if pinned else rng.integers(0, 256, (3, n, pitch), dtype=np.uint8)
    try:
        want = buf.copy()
        rs_ref.c_encode(d, p, want, S=S)
        launches = _timed_launches(enc, lambda: enc.encode_host(buf, S))
        assert launches > 0
        assert np.array_equal(buf[:, :, :S], want[:, :, :S])
        masks = _masks(3, n, p, rng)
        inp = want.copy()
        for g in range(3):
            for r in range(n):
                if not (int(masks[g]) >> r) & 1:
                    inp[g, r, :S] = 0
        buf[:] = inp
        exp = inp.copy()
        rc, st_want = rs_ref.c_reconstruct(d, p, exp, masks, S=S)
        st = np.full(3, -1, np.int8)
        launches = _timed_launches(enc, lambda: enc.reconstruct_host(buf, masks, S, False, st))
        assert launches > 0
        assert np.array_equal(st, st_want)
        assert np.array_equal(buf, exp)
    finally:
        enc.service_stop()
        if pinned:
            fec.host_free(buf.reshape(-1))
        enc.close()


def test_service_restart_while_alive(gpu):
    """stop and restart the service while its block is resident
    (long idle window), many times: a relaunched block must never take the
    stop request still on the mailbox line, nor an older request, for a new
    one -- every call after a restart is served (no launch) with the right
    bytes."""
    d, p, S = 10, 3, 1470
    n, pitch = d + p, 1472
    rng = np.random.default_rng(17)
    enc = fec.New(d, p)
    b = _pinned(1, n, pitch, rng)
    try:
        for i in range(60):
            enc.service_start(idle_us=1_000_000)
            for _ in range(2):
                b[:] = rng.integers(0, 256, b.shape, dtype=np.uint8)
                want = b.copy()
                rs_ref.c_encode(d, p, want, S=S)
                assert _timed_launches(enc, lambda: enc.encode_host(b, S)) == 0, i
                assert np.array_equal(b[:, :, :S], want[:, :, :S]), i
            enc.service_stop()
    finally:
        enc.service_stop()
        fec.host_free(b.reshape(-1))
        enc.close()


def test_service_timeout_waits_for_the_block_to_leave(gpu):
    """a call the service does not answer within the
    watchdog timeout (forced: the block stalls 300 ms per request, timeout 50
    ms) returns ErrHip only after the block has left -- so nothing writes the
    caller's batch after the call returns -- and later calls take the launch
    path with the right bytes; the service can be started again."""
    d, p, S = 10, 3, 1470
    n, pitch = d + p, 1472
    rng = np.random.default_rng(23)
    enc = fec.New(d, p)
    b = _pinned(1, n, pitch, rng)
    try:
        enc.service_config(timeout_ms=50, grace_ms=5000, test_stall_us=300_000)
        enc.service_start(idle_us=1_000_000)
        want = b.copy()
        rs_ref.c_encode(d, p, want, S=S)
        t0 = time.perf_counter()
        with pytest.raises(fec.ErrHip):
            enc.encode_host(b, S)
        el = time.perf_counter() - t0
        assert 0.25 < el < 4.0, el  # the stall ran out and the block left before the call returned
        assert not enc.poisoned
        snap = b.copy()
        time.sleep(0.4)
        assert np.array_equal(b, snap), "the batch changed after the call returned"
        # the block served the request on its way out: its bytes are the right ones
        assert np.array_equal(b[:, :, :S], want[:, :, :S])
        b[:, d:, :] = 0
        assert _timed_launches(enc, lambda: enc.encode_host(b, S)) > 0  # service off: launch path
        assert np.array_equal(b[:, :, :S], want[:, :, :S])
        enc.service_config()  # no stall
        enc.service_start()
        b[:, d:, :] = 0
        assert _timed_launches(enc, lambda: enc.encode_host(b, S)) == 0
        assert np.array_equal(b[:, :, :S], want[:, :, :S])
    finally:
        enc.service_stop()
        fec.host_free(b.reshape(-1))
        enc.close()


def test_service_block_that_never_leaves_poisons_the_context(gpu):
    """A block still resident after the grace period (stall 1.2 s, timeout 50
    ms, grace 100 ms): the call fails, the context is poisoned, every later
    call on it fails without touching the GPU, and destroy frees nothing the
    block reads (it finishes later, serving into the batch this test keeps
    alive, and leaves on the stop request)."""
    import torch

    d, p, S = 10, 3, 1470
    n, pitch = d + p, 1472
    rng = np.random.default_rng(29)
    enc = fec.New(d, p)
    b = _pinned(1, n, pitch, rng)
    try:
        enc.service_config(timeout_ms=50, grace_ms=100, test_stall_us=1_200_000)
        enc.service_start(idle_us=1_000_000)
        with pytest.raises(fec.ErrHip):
            enc.encode_host(b, S)
        assert enc.poisoned
        for call in (lambda: enc.encode_host(b, S), lambda: enc.service_start(),
                     lambda: enc.encode_batch(torch.zeros((2, n, pitch), dtype=torch.uint8, device="cuda"), S),
                     lambda: enc.reconstruct_host(b, np.full(1, (1 << n) - 1, np.uint64), S)):
            with pytest.raises(fec.ErrHip):
                call()
        t0 = time.perf_counter()
        enc.close()  # leaks the mailbox and tables: the block still reads them
        el = time.perf_counter() - t0
        # destroy of a poisoned context must not wait for the block
        # (every hipFree / hipHostFree / stream destroy would synchronize with it)
        assert el < 0.5, f"destroy of a poisoned context blocked for {el:.3f} s"
        time.sleep(1.6)  # the stalled block serves, sees the stop line and leaves
        torch.cuda.synchronize()
    finally:
        fec.host_free(b.reshape(-1))


def test_service_block_does_not_hold_other_streams(gpu):
    """A resident block (1-s idle window) must not delay work on other streams:
    its stream has a hardware queue of its own (create_service_stream).  Before
    that, an ordinary stream that HIP's queue pool put on the service's queue
    waited out the idle window -- a staged host encode on another context took
    ~1 s instead of ~2 ms (tools/svc_sync_probe.cpp,
    profiles/r4/svc_sync_probe_queue_ab.jsonl).  Device-wide synchronizes
    (hipFree, torch.cuda.synchronize) still wait for the block, as documented."""
    import torch

    d, p, S = 10, 3, 1350
    n, pitch = d + p, 1360
    rng = np.random.default_rng(17)
    svc, work = fec.New(d, p), fec.New(d, p)
    one = _pinned(1, n, 1472, rng)
    big = _pinned(8192, n, pitch, rng)  # 145 MB: past the zero-copy size, the staged 3-stream pipeline
    try:
        want = big.copy()
        rs_ref.c_encode(d, p, want[:64], S=S)
        work.encode_host(big, S)  # staging and streams allocated before the block is resident
        x = torch.zeros(4, device="cuda")
        x.add_(1)  # torch's kernel loaded before the block is resident
        torch.cuda.synchronize()
        svc.service_start(idle_us=1_000_000)
        svc.encode_host(one, 1470)  # served: the block is resident for the next second
        t0 = time.perf_counter()
        work.encode_host(big, S)
        host_ms = (time.perf_counter() - t0) * 1e3
        worst = 0.0
        for _ in range(8):
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                t0 = time.perf_counter()
                x.add_(1)
                s.synchronize()
                worst = max(worst, (time.perf_counter() - t0) * 1e3)
        svc.encode_host(one, 1470)
        assert host_ms < 300, f"staged host encode waited for the service block: {host_ms:.1f} ms"
        assert worst < 300, f"a fresh stream waited for the service block: {worst:.1f} ms"
        assert np.array_equal(big[:64, :, :S], want[:64, :, :S])
    finally:
        svc.service_stop()
        fec.host_free(one.reshape(-1))
        fec.host_free(big.reshape(-1))
        svc.close()
        work.close()


def test_service_more_contexts_than_hardware_queues(gpu):
    """six contexts (one per connection) start the service and are
    called continuously from six threads -- more than the GPU_MAX_HW_QUEUES (4)
    high-priority queues the service streams come from.  No call times out, no
    context is poisoned, every parity is the oracle's; at most four contexts
    hold a resident block at once (a pool stream each), the others are served
    on the launch path."""
    import threading
    d, p, S = 10, 3, 1470
    n, pitch = d + p, 1472
    nctx, calls = 6, 120
    errors, served = [], []
    ready = threading.Barrier(nctx)

    def worker(seed):
        enc, b = None, None
        try:
            rng = np.random.default_rng(seed)
            enc = fec.New(d, p)
            enc.service_config(timeout_ms=2000, grace_ms=2000)
            b = _pinned(1, n, pitch, rng)
            ready.wait(timeout=60)
            enc.service_start(idle_us=1_000_000)
            hits = 0
            for i in range(calls):
                b[:] = rng.integers(0, 256, b.shape, dtype=np.uint8)
                want = b.copy()
                rs_ref.c_encode(d, p, want, S=S)
                hits += _timed_launches(enc, lambda: enc.encode_host(b, S)) == 0
                if not np.array_equal(b[:, :, :S], want[:, :, :S]):
                    errors.append((seed, i, "bytes"))
                    return
            if enc.poisoned:
                errors.append((seed, "poisoned"))
            served.append(hits >= calls // 2)  # the block's own (re)launches are timed launches too
        except Exception as ex:  # pragma: no cover - reported below
            errors.append((seed, repr(ex)))
        finally:
            if enc is not None:
                enc.service_stop()
                enc.close()
            if b is not None:
                fec.host_free(b.reshape(-1))

    ts = [threading.Thread(target=worker, args=(100 + k,)) for k in range(nctx)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not any(t.is_alive() for t in ts)
    assert not errors, errors
    assert len(served) == nctx
    assert 1 <= sum(served) <= 3, served


_QUEUE_PROBE = r"""
import ctypes, sys
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
from ugo_amd import fec
d, p, G, n, slot = 10, 3, 512, 13, 1488
tx = fec.New(d, p)
pk = fec.host_alloc(G * d * slot).reshape(G * d, slot); pk[:] = 1
ln = fec.host_alloc(G * d * 2).view(np.uint16); ln[:] = 1476
wire = fec.host_alloc(G * n * slot).reshape(G * n, slot)
wl = fec.host_alloc(G * n * 2).view(np.uint16)
tx.tx_assemble_host(pk, ln, wire, wl, max_len=1476)   # the default low-priority copy queue
encs, bufs = [], []
for k in range(6):                                    # more service contexts than the pool holds
    e = fec.New(d, p)
    e.service_start(idle_us=200000)
    b = fec.host_alloc(n * 1472).reshape(1, n, 1472)
    e.encode_host(b, 1470)
    encs.append(e); bufs.append(b)
for s in [torch.cuda.Stream() for _ in range(6)]:     # ordinary streams of the application
    with torch.cuda.stream(s):
        torch.ones(16, device="cuda").sum()
torch.cuda.synchronize()
for e in encs:
    e.service_stop(); e.close()
tx.close()
print("done")
"""


def test_process_hw_queue_footprint(gpu, tmp_path):
    """The library keeps the process within 8 hardware queues (past 8 the GPU's
    scheduler time-slices them, and a resident service block then cost
    concurrent work ~33 %): host TX with the default
    low-priority copy queue, six contexts starting the per-call service, six
    ordinary torch streams -- HIP's own queue log (AMD_LOG_LEVEL=3, in a child
    process) shows at most 8 distinct hardware queues, one low-priority, at
    most 3 high-priority."""
    import os
    import re
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "probe.py"
    script.write_text(_QUEUE_PROBE)
    env = dict(os.environ, AMD_LOG_LEVEL="3", GPU_MAX_HW_QUEUES="4")
    r = subprocess.run([sys.executable, str(script), root], capture_output=True, text=True, env=env, timeout=180)
    assert r.returncode == 0 and "done" in r.stdout, r.stderr[-2000:]
    hw = {}
    for m in re.finditer(r"to map on HWq=(0x[0-9a-f]+) with size \d+ with priority (\d)", r.stderr + r.stdout):
        hw.setdefault(m.group(1), m.group(2))
    assert hw, "no queue creation in HIP's log (log format changed?)"
    prio = [v for v in hw.values()]
    assert len(hw) <= 8, (len(hw), sorted(prio))
    assert prio.count("0") == 1 and prio.count("2") <= 3, sorted(prio)
