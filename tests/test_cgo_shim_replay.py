"""The cgo shim's exact C-ABI call sequence, replayed through ctypes.

INTEGRATION.md §2 holds the Go package a ugo maintainer adds: `ugofec.New`,
`Encode`, `Reconstruct`, `ReconstructData`, replacing klauspost's encoder at
/root/reference/ugo/fec.go:21,59 (New), :202 (Reconstruct) and :238 (Encode).
There is no Go toolchain here, so `GoShim` below transliterates that Go code
statement by statement -- the same C calls, in the same order, with the same
arguments (one pinned staging buffer reused across calls, rows at the 16-B
pitch P = (S+15) &^ 15, groups = 1) -- and the tests check it against the
oracle at ugo's two shard sizes: 1470 (the calcECC window data[k][6:1476],
ugo/fec.go:228-243) and 1476 (input's pool buffers, maxPacketSize,
ugo/constants.go:29).  Through ugo_fec_timing_* every call is checked to run a
16-B vector kernel: no UGO_FEC_KERNEL_BYTES launch (the byte kernel a pitch-S
staging would have taken).  Oracle = checker only.
"""
import ctypes

import numpy as np
import pytest

import rs_ref
from ugo_amd import fec

pytestmark = pytest.mark.gpu

UGO_FEC_OK = 0
UGO_FEC_RECONSTRUCT_DATA_ONLY = 1
UGO_FEC_KERNEL_BYTES = 4


class ShimError(Exception):
    def __init__(self, st):
        super().__init__(fec.strerror(st))
        self.status = st


def status_err(st):  # statusErr
    if st != UGO_FEC_OK:
        raise ShimError(st)


def pitch(S):  # func pitch(S int) int { return (S + 15) &^ 15 }
    return (S + 15) & ~15


class GoShim:
    """package ugofec, line for line."""

    def __init__(self, data_shards, parity_shards):  # func New
        self.lib = lib = fec.load_library()
        assert lib.ugo_fec_abi_version() == 9  # C.UGO_FEC_ABI_VERSION of the header
        ctx = ctypes.c_void_p()
        status_err(lib.ugo_fec_create(0, data_shards, parity_shards, ctypes.byref(ctx)))
        self.ctx, self.d, self.p = ctx, data_shards, parity_shards
        self.stage, self.stageN = ctypes.c_void_p(), 0

    def close(self):  # func (e *Encoder) Close
        poisoned = self.lib.ugo_fec_poisoned(self.ctx) != 0
        self.lib.ugo_fec_destroy(self.ctx)
        if self.stage and not poisoned:
            self.lib.ugo_fec_host_free(self.stage)

    def ServiceStart(self, idle_us):  # func (e *Encoder) ServiceStart(idleUs uint) error
        status_err(self.lib.ugo_fec_service_start(self.ctx, idle_us))

    def staging(self, n):  # func (e *Encoder) staging(n int) []byte
        if n > self.stageN:
            if self.stage:
                self.lib.ugo_fec_host_free(self.stage)
            self.lib.ugo_fec_host_alloc(n, ctypes.byref(self.stage))
            self.stageN = n
        return (ctypes.c_uint8 * n).from_address(self.stage.value)

    def check(self, shards, nil_ok):  # func (e *Encoder) check
        n = self.d + self.p
        if len(shards) != n:
            raise ShimError(3)  # ErrTooFewShards
        lens = (ctypes.c_size_t * n)(*[0 if s is None else len(s) for s in shards])
        size = ctypes.c_size_t(0)
        status_err(self.lib.ugo_fec_check_shards(n, ctypes.cast(lens, ctypes.c_void_p), 1 if nil_ok else 0,
                                                 ctypes.byref(size)))
        return size.value

    def Encode(self, shards):  # func (e *Encoder) Encode(shards [][]byte) error
        S = self.check(shards, False)
        n, P = self.d + self.p, pitch(S)
        buf = self.staging(n * P)
        mv = memoryview(buf).cast("B")
        for k in range(self.d):
            mv[k * P:k * P + S] = shards[k]
        status_err(self.lib.ugo_fec_encode_host(self.ctx, self.stage, 1, S, P))
        for k in range(self.d, n):
            shards[k][:] = mv[k * P:k * P + S]

    def _reconstruct(self, shards, flags):  # func (e *Encoder) reconstruct
        S = self.check(shards, True)
        n, P = self.d + self.p, pitch(S)
        buf = self.staging(n * P)
        mv = memoryview(buf).cast("B")
        mask = (ctypes.c_uint64 * 4)()
        for r, s in enumerate(shards):
            if s is not None and len(s) != 0:
                mask[r // 64] |= 1 << (r % 64)
                mv[r * P:r * P + S] = s
        status = ctypes.c_int8(0)
        status_err(self.lib.ugo_fec_reconstruct_host(self.ctx, self.stage, ctypes.cast(mask, ctypes.c_void_p), 1,
                                                     S, P, flags, ctypes.byref(status)))
        limit = self.d if flags & UGO_FEC_RECONSTRUCT_DATA_ONLY else n
        for r in range(limit):
            if shards[r] is not None and len(shards[r]) != 0:
                continue
            shards[r] = bytearray(mv[r * P:r * P + S])

    def Reconstruct(self, shards):
        self._reconstruct(shards, 0)

    def ReconstructData(self, shards):
        self._reconstruct(shards, UGO_FEC_RECONSTRUCT_DATA_ONLY)

    # measurement hooks (not part of the Go shim): which kernels ran
    def timing_begin(self):
        status_err(self.lib.ugo_fec_timing_begin(self.ctx, 4096))

    def timing_end(self):
        out = np.zeros(4096, fec.LAUNCH_TIME_DTYPE)
        n, untimed = ctypes.c_size_t(), ctypes.c_size_t()
        status_err(self.lib.ugo_fec_timing_end(self.ctx, out.ctypes.data, 4096, ctypes.byref(n),
                                               ctypes.byref(untimed)))
        assert untimed.value == 0
        return out[:n.value]


def _oracle_encode(d, p, data, S):
    g = np.zeros((1, d + p, S), np.uint8)
    for k in range(d):
        g[0, k] = np.frombuffer(bytes(data[k]), np.uint8)
    rs_ref.c_encode(d, p, g)
    return [bytes(g[0, k]) for k in range(d + p)]


@pytest.mark.parametrize("S", [1470, 1476])
def test_shim_encode_reconstruct_vs_oracle(gpu, S):
    d, p, n = 10, 3, 13
    shim = GoShim(d, p)
    rng = np.random.default_rng(S)
    try:
        shim.timing_begin()
        for trial in range(24):
            data = [bytearray(rng.integers(0, 256, S, dtype=np.uint8).tobytes()) for _ in range(d)]
            shards = data + [bytearray(S) for _ in range(p)]
            shim.Encode(shards)
            want = _oracle_encode(d, p, data, S)
            assert [bytes(s) for s in shards] == want, trial
            # Reconstruct: up to p lost shards anywhere, nil or empty as ugo passes them
            e = int(rng.integers(1, p + 1))
            lost = sorted(rng.choice(n, e, replace=False).tolist())
            work = [bytearray(s) for s in shards]
            for r in lost:
                work[r] = None if rng.random() < 0.5 else bytearray()
            shim.Reconstruct(work)
            assert [bytes(s) for s in work] == want, (trial, lost)
            # ReconstructData: data rows back, lost parity rows stay empty
            work = [bytearray(s) for s in shards]
            for r in lost:
                work[r] = None
            shim.ReconstructData(work)
            for r in range(n):
                if r < d or r not in lost:
                    assert bytes(work[r]) == want[r], (trial, r)
                else:
                    assert work[r] is None, (trial, r)
        recs = shim.timing_end()
        kinds = set(int(k) for k in recs["kernel"])
        assert len(recs) >= 24 * 2
        assert UGO_FEC_KERNEL_BYTES not in kinds, "a call ran the byte-granular kernel"
        assert kinds <= {1, 2}, kinds
    finally:
        shim.close()


def test_shim_errors_like_klauspost(gpu):
    """The errors the shim maps back to klauspost's (ugo/fec.go logs and
    swallows them, :60-63, :208-210, :239-241)."""
    d, p, S = 10, 3, 1470
    shim = GoShim(d, p)
    try:
        with pytest.raises(ShimError) as ei:
            shim.Encode([bytearray(S)] * (d + p - 1))
        assert ei.value.status == 3  # ErrTooFewShards
        bad = [bytearray(S) for _ in range(d + p)]
        bad[4] = bytearray(S - 1)
        with pytest.raises(ShimError) as ei:
            shim.Encode(bad)
        assert ei.value.status == 5  # ErrShardSize
        with pytest.raises(ShimError) as ei:
            shim.Encode([bytearray() for _ in range(d + p)])
        assert ei.value.status == 4  # ErrShardNoData
        few = [bytearray(S) for _ in range(d + p)]
        for r in (0, 3, 7, 11):
            few[r] = None
        with pytest.raises(ShimError) as ei:
            shim.Reconstruct(few)
        assert ei.value.status == 3  # ErrTooFewShards: p + 1 lost
        assert few[0] is None  # nothing filled in
    finally:
        shim.close()
