"""The cgo shim's exact C-ABI call sequence, replayed through ctypes.

go/ugofec/ugofec.go is the Go package a ugo maintainer adds (go/fec.go.patch
is the edit to ugo/fec.go): `ugofec.New`, `Encode`, `Reconstruct`,
`ReconstructData`, replacing klauspost's encoder at
/root/reference/ugo/fec.go:21,59 (New), :202 (Reconstruct) and :238 (Encode),
plus the batch paths `RecoverRing` (ugo_fec_rx_recover_host) and `AssembleTx`
(ugo_fec_tx_assemble_host).  There is no Go toolchain here, so `GoShim` below
transliterates that Go code statement by statement -- the same C calls, in the
same order, with the same arguments (one pinned staging buffer reused across
calls, rows at the 16-B pitch P = (S+15) &^ 15, groups = 1) -- and the tests
check it against the oracle at ugo's two shard sizes: 1470 (the calcECC window
data[k][6:1476], ugo/fec.go:228-243) and 1476 (input's pool buffers,
maxPacketSize, ugo/constants.go:29).  Through ugo_fec_timing_* every call is
checked to run a 16-B vector kernel: no UGO_FEC_KERNEL_BYTES launch (the byte
kernel a pitch-S staging would have taken).  A CPU test parses the .go file
and checks that every C.ugo_fec_* call in it is one GoShim replays, declared
in include/ugo_fec.h.  Oracle = checker only.
"""
import ctypes
import inspect
import os
import re
import shutil
import subprocess
import tempfile

import numpy as np
import pytest

import rc4_ref
import rs_ref
from ugo_amd import fec

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO_SHIM = os.path.join(ROOT, "go", "ugofec", "ugofec.go")
GO_PATCH = os.path.join(ROOT, "go", "fec.go.patch")

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
    """package ugofec (go/ugofec/ugofec.go), line for line."""

    def statusErr(self, st):  # func statusErr(st C.int) error: klauspost's errors 1-5, else the library's text
        if st != UGO_FEC_OK:
            err = ShimError(st)
            if st > 5:
                err.args = (self.lib.ugo_fec_strerror(st).decode(),)
            raise err

    def __init__(self, data_shards, parity_shards):  # func New
        self.lib = lib = fec.load_library()
        assert lib.ugo_fec_abi_version() == 9  # C.UGO_FEC_ABI_VERSION of the header
        ctx = ctypes.c_void_p()
        self.statusErr(lib.ugo_fec_create(0, data_shards, parity_shards, ctypes.byref(ctx)))
        self.ctx, self.d, self.p = ctx, data_shards, parity_shards
        self.stage, self.stageN = ctypes.c_void_p(), 0

    def close(self):  # func (e *Encoder) Close
        poisoned = self.lib.ugo_fec_poisoned(self.ctx) != 0
        self.lib.ugo_fec_destroy(self.ctx)
        if self.stage and not poisoned:
            self.lib.ugo_fec_host_free(self.stage)

    def ServiceStart(self, idle_us):  # func (e *Encoder) ServiceStart(idleUs uint) error
        self.statusErr(self.lib.ugo_fec_service_start(self.ctx, idle_us))

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
        self.statusErr(self.lib.ugo_fec_check_shards(n, ctypes.cast(lens, ctypes.c_void_p), 1 if nil_ok else 0,
                                                 ctypes.byref(size)))
        return size.value

    def Encode(self, shards):  # func (e *Encoder) Encode(shards [][]byte) error
        S = self.check(shards, False)
        n, P = self.d + self.p, pitch(S)
        buf = self.staging(n * P)
        mv = memoryview(buf).cast("B")
        for k in range(self.d):
            mv[k * P:k * P + S] = shards[k]
        self.statusErr(self.lib.ugo_fec_encode_host(self.ctx, self.stage, 1, S, P))
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
        self.statusErr(self.lib.ugo_fec_reconstruct_host(self.ctx, self.stage, ctypes.cast(mask, ctypes.c_void_p), 1,
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

    # ---- batch paths
    def HostAlloc(self, n):  # func HostAlloc(n int) ([]byte, error)
        p = ctypes.c_void_p()
        self.statusErr(self.lib.ugo_fec_host_alloc(n, ctypes.byref(p)))
        return np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(p.value))

    def HostFree(self, b):  # func HostFree(b []byte)
        if len(b) != 0:
            self.lib.ugo_fec_host_free(ctypes.c_void_p(b.ctypes.data))

    def RecoverRing(self, ring, slot, lens, pad, first_group, groups, shard_size, out, out_stride, index):
        npk, max_out = len(lens), len(index)
        if max_out > 0 and out.nbytes < (max_out - 1) * out_stride + shard_size:
            raise ValueError("ugofec: out holds fewer than len(index) shards")
        if npk > 0 and ring.nbytes < npk * slot:
            raise ValueError("ugofec: ring holds fewer than len(lens) slots")
        stats = np.zeros(5, np.uint32)
        n_out = ctypes.c_size_t(0)
        st = self.lib.ugo_fec_rx_recover_host(
            self.ctx, ring.ctypes.data if ring.size else None, slot, lens.ctypes.data if npk else None, npk,
            None if pad is None else pad.ctypes.data, first_group, groups, shard_size, None, stats.ctypes.data,
            out.ctypes.data if out.size else None, out_stride, max_out, index.ctypes.data if max_out else None,
            ctypes.byref(n_out))
        self.statusErr(st)
        return n_out.value, stats

    def AssembleTx(self, pkts, slot_in, lens, first_seq, pad, max_len, wire, slot_out, wire_lens, status):
        n = self.d + self.p
        if len(lens) % self.d != 0:
            raise ValueError("ugofec: lens must hold whole groups of d packets")
        groups = len(lens) // self.d
        if groups == 0:
            return
        if (pkts.nbytes < groups * self.d * slot_in or wire.nbytes < groups * n * slot_out
                or len(wire_lens) < groups * n or (status is not None and len(status) < groups)):
            raise ValueError("ugofec: buffer shorter than the batch")
        self.statusErr(self.lib.ugo_fec_tx_assemble_host(
            self.ctx, pkts.ctypes.data, slot_in, lens.ctypes.data, groups, first_seq,
            None if pad is None else pad.ctypes.data, max_len, wire.ctypes.data, slot_out, wire_lens.ctypes.data,
            None if status is None else status.ctypes.data))

    # measurement hooks (not part of the Go shim): which kernels ran
    def timing_begin(self):
        self.statusErr(self.lib.ugo_fec_timing_begin(self.ctx, 4096))

    def timing_end(self):
        out = np.zeros(4096, fec.LAUNCH_TIME_DTYPE)
        n, untimed = ctypes.c_size_t(), ctypes.c_size_t()
        self.statusErr(self.lib.ugo_fec_timing_end(self.ctx, out.ctypes.data, 4096, ctypes.byref(n),
                                               ctypes.byref(untimed)))
        assert untimed.value == 0
        return out[:n.value]


def _oracle_encode(d, p, data, S):
    g = np.zeros((1, d + p, S), np.uint8)
    for k in range(d):
        g[0, k] = np.frombuffer(bytes(data[k]), np.uint8)
    rs_ref.c_encode(d, p, g)
    return [bytes(g[0, k]) for k in range(d + p)]


def _go_c_calls(src):
    """The C.ugo_fec_* functions a Go file calls (comments stripped)."""
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    return set(re.findall(r"\bC\.(ugo_fec_[a-z0-9_]+)\s*\(", src))


def test_go_shim_calls_are_replayed_and_declared():
    """Every C.ugo_fec_* call of go/ugofec/ugofec.go is one GoShim replays (so
    the GPU tests below exercise it) and one include/ugo_fec.h declares; every
    C.UGO_FEC_* constant it names is defined there."""
    go = open(GO_SHIM).read()
    calls = _go_c_calls(go)
    assert {"ugo_fec_create", "ugo_fec_encode_host", "ugo_fec_reconstruct_host", "ugo_fec_rx_recover_host",
            "ugo_fec_tx_assemble_host"} <= calls
    replayed = set(re.findall(r"lib\.(ugo_fec_[a-z0-9_]+)\s*\(", inspect.getsource(GoShim)))
    assert calls <= replayed, f"calls the replay does not make: {sorted(calls - replayed)}"
    declared = set(fec.header_symbols((fec.HEADER_PATH,)))
    assert calls <= declared, sorted(calls - declared)
    header = open(fec.HEADER_PATH).read()
    for const in set(re.findall(r"\bC\.(UGO_FEC_[A-Z0-9_]+)", go)):
        assert re.search(r"\b" + const + r"\b", header), const
    assert 'import "C"' in go and "#cgo CFLAGS: -I${SRCDIR}/../../include" in go


@pytest.mark.skipif(not os.path.exists("/root/reference/ugo/fec.go") or shutil.which("patch") is None,
                    reason="needs the reference tree (build container only) and patch(1)")
def test_fec_go_patch_applies_to_the_reference():
    """go/fec.go.patch applies cleanly to ugo/fec.go and swaps exactly the
    encoder: the klauspost import, the enc field's type, New (ugo/fec.go:9,21,59)."""
    with tempfile.TemporaryDirectory() as td:
        os.makedirs(os.path.join(td, "ugo"))
        shutil.copy("/root/reference/ugo/fec.go", os.path.join(td, "ugo", "fec.go"))
        r = subprocess.run(["patch", "-p1", "-i", GO_PATCH], cwd=td, capture_output=True, text=True)
        assert r.returncode == 0, r.stdout + r.stderr
        out = open(os.path.join(td, "ugo", "fec.go")).read()
    assert "reedsolomon" not in out and "ugofec.New(dataShards, parityShards)" in out
    assert "Reconstruct(shards [][]byte) error" in out


@pytest.mark.gpu
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


@pytest.mark.gpu
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


@pytest.mark.gpu
def test_shim_batch_tx_then_rx_round_trip(gpu):
    """AssembleTx then RecoverRing through the shim's C calls, pinned buffers
    from HostAlloc: 40 groups of 10 full 1476-B data packets, RC4.  The wire
    packets are checked against the oracle (each data packet = header + its
    payload, each parity packet's window [6, 1476) = rs_ref's encode of the
    data windows, ugo/fec.go:228-243), then 1-3 packets per group are lost and
    the ring shuffled: the recovered shards are exactly the lost data packets'
    payloads, in `recovered` order (ugo/fec.go:203-207)."""
    d, p, G, L, slot = 10, 3, 40, 1476, 1488
    n, S = d + p, L - 6
    shim = GoShim(d, p)
    rng = np.random.default_rng(606)
    bufs = []
    try:
        def alloc(nbytes):
            b = shim.HostAlloc(nbytes)
            bufs.append(b)
            return b

        pad = np.frombuffer(rc4_ref.keystream(b"1234567890123456", slot), np.uint8).copy()
        pk = alloc(G * d * slot).reshape(G * d, slot)
        pk[:] = rng.integers(0, 256, pk.shape, dtype=np.uint8)
        lens = alloc(G * d * 2).view(np.uint16)
        lens[:] = L
        wire = alloc(G * n * slot).reshape(G * n, slot)
        wl = alloc(G * n * 2).view(np.uint16)
        st = alloc(G).view(np.int8)
        shim.AssembleTx(pk, slot, lens, 0, pad, L, wire, slot, wl, st)
        assert (st == 0).all() and (wl == L).all()
        plain = wire[:, :L] ^ pad[:L]
        seq = np.arange(G * n, dtype=np.uint32)
        assert np.array_equal(plain[:, :4].copy().view(np.uint32).ravel(), seq)
        flags = plain[:, 4:6].copy().view(np.uint16).ravel()
        assert np.array_equal(flags, np.where(seq % n < d, 0xF1, 0xF2))
        grp = plain.reshape(G, n, L)
        assert np.array_equal(grp[:, :d, 6:], pk.reshape(G, d, slot)[:, :, 6:L])
        want = np.zeros((G, n, S), np.uint8)
        want[:, :d] = grp[:, :d, 6:]
        rs_ref.c_encode(d, p, want)
        assert np.array_equal(grp[:, d:, 6:], want[:, d:])
        # the channel: lose 1-3 packets of each group, shuffle
        keep = np.ones(G * n, bool)
        for g in range(G):
            keep[g * n + rng.choice(n, int(rng.integers(1, p + 1)), replace=False)] = False
        order = rng.permutation(np.nonzero(keep)[0])
        ring = alloc(len(order) * slot).reshape(len(order), slot)
        ring[:] = wire[order]
        rl = alloc(len(order) * 2).view(np.uint16)
        rl[:] = L
        lost = [(g, r) for g in range(G) for r in range(d) if not keep[g * n + r]]
        out = alloc(len(lost) * 1472).reshape(len(lost), 1472)
        index = np.zeros(len(lost), np.uint32)
        nrec, stats = shim.RecoverRing(ring, slot, rl, pad, 0, G, S, out, 1472, index)
        assert nrec == len(lost) and stats.tolist() == [len(order), 0, 0, 0, 0]
        assert index.tolist() == [g * n + r for g, r in lost]
        for j, (g, r) in enumerate(lost):
            assert np.array_equal(out[j, :S], pk[g * d + r, 6:L]), (g, r)
    finally:
        for b in bufs:
            shim.HostFree(b)
        shim.close()
