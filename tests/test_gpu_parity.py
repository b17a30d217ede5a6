"""GPU parity: the gfx950 kernels (through the C-ABI) are bit-exact against the
CPU oracle (oracle/rs_oracle.c) on the same seeded inputs, on the committed
golden fixtures, and -- at BASELINE sizes -- on size-independent properties
(encode -> erase -> reconstruct round trip, linearity).

Oracle = checker only; every result compared here was computed on the GPU.
"""
import os

import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import rs_ref
from ugo_amd import fec

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _rand(G, n, pitch, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randint(0, 256, (G, n, pitch), dtype=torch.uint8, generator=g)


def _dev(x):
    return torch.as_tensor(x).contiguous().cuda()


def _masks_to_dev(masks):
    return torch.as_tensor(np.asarray(masks, dtype=np.uint64).view(np.int64)).cuda()


def _erase(arr, masks, n):
    arr = arr.copy()
    for g, m in enumerate(masks):
        for r in range(n):
            if not (int(m) >> r) & 1:
                arr[g, r] = 0
    return arr


@pytest.fixture(scope="module")
def fx():
    return dict(np.load(os.path.join(GOLD, "fixtures_v1.npz")))


def test_matrix_matches_oracle(gpu):
    for d, p in [(10, 3), (32, 8), (5, 5), (1, 1), (20, 4)]:
        enc = fec.New(d, p)
        assert np.array_equal(enc.matrix(), rs_ref.c_matrix(d, p))


@pytest.mark.parametrize("S,pitch", [(1350, 1360), (1350, 1350), (1476, 1488), (16, 16), (1, 16), (1000, 1024)])
def test_encode_10_3_vs_oracle(gpu, S, pitch):
    d, p, n, G = 10, 3, 13, 777
    host = _rand(G, n, pitch, 1 + S).numpy()
    want = host.copy()
    rs_ref.c_encode(d, p, want, S=S)
    t = _dev(host)
    enc = fec.New(d, p)
    enc.encode_batch(t, shard_size=S)
    torch.cuda.synchronize()
    got = t.cpu().numpy()
    assert np.array_equal(got[:, :, :S], want[:, :, :S])
    assert np.array_equal(got[:, :, S:], host[:, :, S:]), "padding columns must not be written"


def test_golden_fixtures_on_gpu(gpu, fx):
    enc = fec.New(10, 3)
    data = fx["g10_enc_data"]
    t = torch.zeros((data.shape[0], 13, 1360), dtype=torch.uint8)
    t[:, :10, :1350] = torch.as_tensor(data)
    t = t.cuda()
    enc.encode_batch(t, shard_size=1350)
    assert np.array_equal(t.cpu().numpy()[:, 10:, :1350], fx["g10_enc_parity"])
    for key in ("g10", "g10x"):
        src = fx[f"{key}_in"]
        pitch = ((src.shape[2] + 15) // 16) * 16
        t = torch.zeros((src.shape[0], 13, pitch), dtype=torch.uint8)
        t[:, :, :src.shape[2]] = torch.as_tensor(src)
        t = t.cuda()
        st = torch.full((src.shape[0],), -1, dtype=torch.int8, device="cuda")
        enc.reconstruct_batch(t, _masks_to_dev(fx[f"{key}_mask"]), shard_size=src.shape[2], status=st)
        assert np.array_equal(t.cpu().numpy()[:, :, :src.shape[2]], fx[f"{key}_out"])
        assert (st.cpu() == 0).all()
    # jumbo (32+8)x9000, 8 mixed erasures: d+p = 40 > 16 -> per-group device descriptors
    j = fx["g32_out"]
    mk = fx["g32_mask"]
    jin = _erase(j, mk, 40)
    enc32 = fec.New(32, 8)
    t = torch.zeros((1, 40, 9008), dtype=torch.uint8)
    t[:, :, :9000] = torch.as_tensor(jin)
    t = t.cuda()
    enc32.reconstruct_batch(t, _masks_to_dev(mk), shard_size=9000)
    assert np.array_equal(t.cpu().numpy()[:, :, :9000], j)
    # calcECC window (offset 6 -> unaligned base): byte-granular kernel path
    buf = fx["calcecc_in"]
    t = _dev(buf)
    base = t[:, :, 6:]
    lib = fec.load_library()
    rc = lib.ugo_fec_encode(enc._h, base.data_ptr(), 1, 1100 - 6, 1476, fec._stream_handle(None))
    assert rc == 0
    assert np.array_equal(t.cpu().numpy(), fx["calcecc_out"])


def test_reconstruct_every_pattern_10_3(gpu):
    """All 8192 presence masks of a (10+3) group, one group each, in one batch."""
    d, p, n, S, pitch = 10, 3, 13, 1350, 1360
    masks = np.arange(1 << n, dtype=np.uint64)
    G = len(masks)
    host = _rand(G, n, pitch, 5).numpy()
    rs_ref.c_encode(d, p, host, S=S)  # consistent codewords (oracle builds the input only)
    inp = _erase(host, masks, n)
    want = inp.copy()
    rc, want_st = rs_ref.c_reconstruct(d, p, want, masks, S=S)
    t = _dev(inp)
    st = torch.full((G,), -1, dtype=torch.int8, device="cuda")
    enc = fec.New(d, p)
    enc.reconstruct_batch(t, _masks_to_dev(masks), shard_size=S, status=st)
    got = t.cpu().numpy()
    assert np.array_equal(st.cpu().numpy(), want_st)
    assert np.array_equal(got[:, :, :S], want[:, :, :S])
    ok = np.array([bin(int(m)).count("1") >= d for m in masks])
    assert np.array_equal(got[ok][:, :, :S], host[ok][:, :, :S])  # round trip


@pytest.mark.parametrize("table_max", ["16", "0"])
def test_reconstruct_inconsistent_inputs(gpu, table_max, monkeypatch):
    """Rows that are not a codeword (stale pool tails, ugo/fec.go:84-87): output
    depends on the survivor choice, which must be klauspost's (first d present).
    table_max=0 forces the per-group device descriptor path (k_prepare)."""
    monkeypatch.setenv("UGO_FEC_TABLE_MAX_SHARDS", table_max)
    d, p, n, S, pitch = 10, 3, 13, 1350, 1360
    G = 4096
    rng = np.random.default_rng(9)
    host = _rand(G, n, pitch, 9).numpy()
    masks = rng.integers(0, 1 << n, G).astype(np.uint64)
    masks[:64] = (1 << n) - 1  # nothing to do
    want = host.copy()
    rc, want_st = rs_ref.c_reconstruct(d, p, want, masks, S=S)
    t = _dev(host)
    st = torch.full((G,), -1, dtype=torch.int8, device="cuda")
    enc = fec.New(d, p)
    enc.reconstruct_batch(t, _masks_to_dev(masks), shard_size=S, status=st)
    assert np.array_equal(st.cpu().numpy(), want_st)
    assert np.array_equal(t.cpu().numpy(), want)


@pytest.mark.parametrize("d,p,S,pitch", [(4, 2, 100, 112), (5, 5, 64, 64), (12, 4, 333, 336),
                                         (20, 4, 200, 208), (32, 8, 9000, 9008), (3, 1, 50, 50),
                                         (40, 6, 70, 80), (1, 1, 7, 16), (7, 0, 32, 32),
                                         (5, 3, 1500, 1504), (8, 4, 4096, 4096), (16, 4, 1030, 1040),
                                         (56, 8, 256, 256),  # d+p = 64: the widest presence mask
                                         (24, 8, 2040, 2048),  # 128 chunks: k_apply_qa, no idle lane
                                         (40, 8, 2000, 2000),  # d > 32 on the streaming kernels (qa)
                                         (50, 4, 1500, 1504),  # d > 32, 94 chunks: k_apply_q
                                         (48, 16, 1344, 1344)])  # d > 32, p > 8: outputs in passes of 8
def test_generic_geometries(gpu, d, p, S, pitch):
    n = d + p
    G = 300
    host = _rand(G, n, pitch, d * 100 + p).numpy()
    want = host.copy()
    rs_ref.c_encode(d, p, want, S=S)
    enc = fec.New(d, p)
    t = _dev(host)
    enc.encode_batch(t, shard_size=S)
    got = t.cpu().numpy()
    assert np.array_equal(got, want)
    if p == 0:
        return
    rng = np.random.default_rng(d + p)
    masks = np.zeros(G, np.uint64)
    for g in range(G):
        e = int(rng.integers(0, p + 2))  # includes too-few-shards groups
        er = rng.choice(n, size=min(e, n), replace=False)
        m = (1 << n) - 1
        for r in er:
            m &= ~(1 << int(r))
        masks[g] = m
    inp = _erase(got, masks, n)
    want2 = inp.copy()
    rc, want_st = rs_ref.c_reconstruct(d, p, want2, masks, S=S)
    for data_only in (False, True):
        want3 = inp.copy()
        rs_ref.c_reconstruct(d, p, want3, masks, S=S, data_only=data_only)
        t = _dev(inp)
        st = torch.full((G,), -1, dtype=torch.int8, device="cuda")
        enc.reconstruct_batch(t, _masks_to_dev(masks), shard_size=S, data_only=data_only, status=st)
        assert np.array_equal(st.cpu().numpy(), want_st)
        assert np.array_equal(t.cpu().numpy(), want3), (d, p, data_only)


def test_full_size_round_trip_and_linearity(gpu):
    """BASELINE configs[1]/[2] size: 65536 groups (10+3)x1350, 2 random erasures."""
    d, p, n, S, pitch, G = 10, 3, 13, 1350, 1360, 65536
    enc = fec.New(d, p)
    a = torch.randint(0, 256, (G, n, pitch), dtype=torch.uint8, device="cuda")
    b = torch.randint(0, 256, (G, n, pitch), dtype=torch.uint8, device="cuda")
    ab = a ^ b
    for x in (a, b, ab):
        enc.encode_batch(x, shard_size=S)
    assert torch.equal((a ^ b)[:, :, :S], ab[:, :, :S])  # GF linearity
    ref = a.clone()
    gen = torch.Generator(device="cpu").manual_seed(2)
    e1 = torch.randint(0, n, (G,), generator=gen)
    e2 = (e1 + torch.randint(1, n, (G,), generator=gen)) % n
    masks = ((1 << n) - 1) ^ (1 << e1) ^ (1 << e2)
    masks = masks.to(torch.int64).cuda()
    gi = torch.arange(G, device="cuda")
    a[gi, e1.cuda()] = 0
    a[gi, e2.cuda()] = 0
    enc.reconstruct_batch(a, masks, shard_size=S)
    assert torch.equal(a[:, :, :S], ref[:, :, :S])
    # spot-check a sample against the oracle too
    idx = torch.randint(0, G, (64,), generator=gen)
    sample = ref[idx.cuda()].cpu().numpy().copy()
    want = sample.copy()
    want[:, d:] = 0
    rs_ref.c_encode(d, p, want, S=S)
    assert np.array_equal(sample[:, :, :S], want[:, :, :S])


def test_full_size_timed_form_vs_oracle(gpu):
    """The exact form bench.py times (BASELINE configs[1]+[2]): planar
    [13][65536][1360] batch, encode, then reconstruct_into a separate
    [3][65536][1360] output with 2 uniformly random erasures per group
    (bench.make_masks).  Full-size round trip, plus 512 groups checked byte for
    byte against the oracle (encode and reconstruct), the output slots past the
    erasures untouched and the input never written."""
    import bench

    d, p, n, S, pitch, G = 10, 3, 13, 1350, 1360, 65536
    enc = fec.New(d, p)
    gen = torch.Generator(device="cuda").manual_seed(0x5EED)
    sh = torch.randint(0, 256, (n, G, pitch), dtype=torch.uint8, device="cuda", generator=gen)
    host0 = sh.cpu().numpy()
    enc.encode_batch(sh, shard_size=S, shard_major=True)
    masks, erased = bench.make_masks(G, n, 2, 0x5EED + 1000, "cuda")
    view = sh.transpose(0, 1)
    full = view.clone()
    gi = torch.arange(G, device="cuda")
    for j in range(2):
        view[gi, erased[:, j].cuda()] = 0
    before = sh.clone()
    out = torch.full((p, G, pitch), 0xA5, dtype=torch.uint8, device="cuda")
    st = torch.full((G,), -1, dtype=torch.int8, device="cuda")
    enc.reconstruct_into(sh, masks, out, shard_size=S, status=st, shard_major=True)
    torch.cuda.synchronize()
    assert torch.equal(sh, before), "reconstruct_into wrote its input"
    assert bool((st == 0).all())
    es = erased.sort(dim=1).values.cuda()
    for j in range(2):  # the full round trip
        assert torch.equal(out[j, :, :S], full[gi, es[:, j], :S])
    assert bool((out[2] == 0xA5).all()), "slot past the erasures written"
    # oracle sample: 512 groups spread over the batch
    idx = np.sort(np.random.default_rng(3).choice(G, 512, replace=False))
    smp = np.ascontiguousarray(host0.transpose(1, 0, 2)[idx][:, :, :S])
    rs_ref.c_encode(d, p, smp)
    got_full = full[torch.as_tensor(idx).cuda()].cpu().numpy()[:, :, :S]
    assert np.array_equal(got_full, smp), "encode differs from the oracle"
    m = masks.cpu().numpy().view(np.uint64)[idx]
    inp = _erase(smp, m, n)
    want = inp.copy()
    rc, want_st = rs_ref.c_reconstruct(d, p, want, m)
    assert rc == 0 and not want_st.any()
    o = out.cpu().numpy()[:, idx, :S]
    er = es.cpu().numpy()[idx]
    for k in range(len(idx)):
        for j in range(2):
            assert np.array_equal(o[j, k], want[k, er[k, j]]), (idx[k], j)


def test_go_shaped_api(gpu):
    enc = fec.New(10, 3)
    rng = np.random.default_rng(4)
    shards = [bytearray(rng.integers(0, 256, 1350, dtype=np.uint8).tobytes()) for _ in range(10)] + \
             [bytearray(1350) for _ in range(3)]
    enc.Encode(shards)
    ref = [bytes(s) for s in shards]
    want = np.array([list(s) for s in ref], np.uint8)[None].copy()
    w2 = want.copy()
    w2[:, 10:] = 0
    rs_ref.c_encode(10, 3, w2)
    assert np.array_equal(w2, want)
    lost = list(shards)
    lost[2] = None
    lost[11] = bytearray()
    enc.Reconstruct(lost)
    assert [bytes(s) for s in lost] == ref
    lost = list(ref)
    lost = [bytearray(s) for s in lost]
    lost[0] = lost[1] = lost[12] = None
    enc.ReconstructData(lost)
    assert bytes(lost[0]) == ref[0] and bytes(lost[1]) == ref[1] and lost[12] is None
    with pytest.raises(fec.ErrTooFewShards):
        enc.Reconstruct([None] * 4 + [bytearray(ref[i]) for i in range(4, 13)])
    with pytest.raises(fec.ErrTooFewShards):
        enc.Encode(shards[:12])
    with pytest.raises(fec.ErrShardSize):
        enc.Encode(shards[:12] + [bytearray(10)])
    with pytest.raises(fec.ErrShardNoData):
        enc.Reconstruct([None] * 13)


def test_host_api_pipelined(gpu):
    """Host buffers staged through the engine's H2D -> kernel -> D2H pipeline,
    several chunks (jumbo groups: ~180 groups per 64 MiB staging buffer)."""
    d, p, n, S, pitch, G = 32, 8, 40, 9000, 9008, 600
    host = _rand(G, n, pitch, 77).numpy()
    want = host.copy()
    rs_ref.c_encode(d, p, want, S=S)
    enc = fec.New(d, p)
    got = host.copy()
    enc.encode_host(got, S)
    assert np.array_equal(got, want)
    rng = np.random.default_rng(5)
    masks = np.array([((1 << n) - 1) & ~int(sum(1 << int(r) for r in rng.choice(n, int(rng.integers(0, 9)),
                                                                                 replace=False)))
                      for _ in range(G)], dtype=np.uint64)
    inp = _erase(want, masks, n)
    st = np.full(G, -1, np.int8)
    out = inp.copy()
    assert enc.reconstruct_host(out, masks, S, status=st) == 0
    assert (st == 0).all()
    assert np.array_equal(out[:, :, :S], want[:, :, :S])
    assert np.array_equal(out[:, :, S:], inp[:, :, S:]), "padding bytes must be untouched"
    # pinned buffer variant
    buf = fec.host_alloc(G * n * pitch)
    try:
        arr = buf.reshape(G, n, pitch)
        arr[:] = inp
        assert enc.reconstruct_host(arr, masks, S) == 0
        assert np.array_equal(arr[:, :, :S], want[:, :, :S])
    finally:
        fec.host_free(buf)


def test_host_staged_paths_after_copy_queue_toggle(gpu):
    """ugo_fec_set_host_copy_queue drops the H2D stream; the staged encode_host /
    reconstruct_host paths that follow (pageable batches, >= 3 chunks, so a
    chunk runs on that stream) make it again instead of falling back to the
    legacy null stream, with results equal to the oracle's in
    every state of the switch."""
    d, p, n, S, pitch, G = 10, 3, 13, 1350, 1360, 8000  # 64-MiB stages: 3,795 groups each -> 3 chunks
    host = _rand(G, n, pitch, 79).numpy()
    want = host.copy()
    rs_ref.c_encode(d, p, want, S=S)
    rng = np.random.default_rng(9)
    masks = np.array([((1 << n) - 1) & ~int(sum(1 << int(r) for r in rng.choice(n, int(rng.integers(0, 4)),
                                                                                 replace=False)))
                      for _ in range(G)], dtype=np.uint64)
    inp = _erase(want, masks, n)
    enc = fec.New(d, p)
    for on in (False, True, True, False):
        enc.set_host_copy_queue(on)
        got = host.copy()
        enc.encode_host(got, S)
        assert np.array_equal(got, want), on
        out = inp.copy()
        assert enc.reconstruct_host(out, masks, S) == 0
        assert np.array_equal(out[:, :, :S], want[:, :, :S]), on


@pytest.mark.parametrize("offset,pitch,data_only", [(256, 1360, False), (3, 1353, False), (16, 1360, True)])
def test_host_reconstruct_pinned_zero_copy(gpu, offset, pitch, data_only):
    """Pinned host batches are reconstructed zero-copy: the kernels read the
    survivors and write only the erased rows through the batch's mapping -- at an interior
    pointer of the allocation, 16-B aligned (vector form) or not (byte form),
    with failing groups left untouched and DATA_ONLY leaving parity rows."""
    d, p, n, S, G = 10, 3, 13, 1350, 700
    host = _rand(G, n, pitch, 91 + offset).numpy()
    want = host.copy()
    rs_ref.c_encode(d, p, want, S=S)
    rng = np.random.default_rng(offset)
    masks = []
    for g in range(G):
        k = int(rng.integers(0, p + 2)) if g % 50 else p + 1  # every 50th group: too few shards
        masks.append(((1 << n) - 1) & ~int(sum(1 << int(r) for r in rng.choice(n, k, replace=False))))
    masks = np.array(masks, dtype=np.uint64)
    inp = want.copy()
    for g, m in enumerate(masks):
        for r in range(n):
            if not (int(m) >> r) & 1:
                inp[g, r, :S] = rng.integers(0, 256, S, dtype=np.uint8)  # garbage in erased rows
    enc = fec.New(d, p)
    buf = fec.host_alloc(G * n * pitch + 4096)
    try:
        arr = buf[offset:offset + G * n * pitch].reshape(G, n, pitch)
        arr[:] = inp
        st = np.full(G, -1, np.int8)
        agg = enc.reconstruct_host(arr, masks, S, data_only=data_only, status=st)
        ok = np.array([bin(int(m)).count("1") >= d for m in masks])
        assert (st[ok] == 0).all() and (st[~ok] != 0).all() and agg == st[~ok][0]
        got = arr.copy()
    finally:
        fec.host_free(buf)
    assert np.array_equal(got[~ok], inp[~ok]), "failing groups must be untouched"
    assert np.array_equal(got[:, :, S:], inp[:, :, S:]), "padding bytes must be untouched"
    if data_only:
        assert np.array_equal(got[ok][:, :d, :S], want[ok][:, :d, :S])
        assert np.array_equal(got[ok][:, d:, :S], inp[ok][:, d:, :S]), "DATA_ONLY must leave parity rows"
    else:
        assert np.array_equal(got[ok][:, :, :S], want[ok][:, :, :S])


@pytest.mark.parametrize("d,p,S,pitch", [(10, 3, 1350, 1360), (32, 8, 9000, 9008), (6, 2, 77, 80),
                                         (10, 3, 1350, 1350), (10, 3, 1476, 1476), (5, 2, 333, 333)])
def test_shard_major_layout(gpu, d, p, S, pitch):
    """Planar [d+p][G][pitch] batches (ugo_fec_*_strided) give the same bytes."""
    n, G = d + p, 513
    host = _rand(G, n, pitch, 31 + d).numpy()
    want = host.copy()
    rs_ref.c_encode(d, p, want, S=S)
    enc = fec.New(d, p)
    t = _dev(np.ascontiguousarray(host.transpose(1, 0, 2)))
    enc.encode_batch(t, shard_size=S, shard_major=True)
    got = t.cpu().numpy().transpose(1, 0, 2)
    assert np.array_equal(got, want)
    rng = np.random.default_rng(3)
    masks = np.array([((1 << n) - 1) & ~int(sum(1 << int(r) for r in rng.choice(n, int(rng.integers(0, p + 2)),
                                                                                 replace=False)))
                      for _ in range(G)], dtype=np.uint64)
    inp = _erase(want, masks, n)
    want2 = inp.copy()
    rc, want_st = rs_ref.c_reconstruct(d, p, want2, masks, S=S)
    t = _dev(np.ascontiguousarray(inp.transpose(1, 0, 2)))
    st = torch.full((G,), -1, dtype=torch.int8, device="cuda")
    enc.reconstruct_batch(t, _masks_to_dev(masks), shard_size=S, status=st, shard_major=True)
    assert np.array_equal(st.cpu().numpy(), want_st)
    assert np.array_equal(t.cpu().numpy().transpose(1, 0, 2), want2)


def test_empty_batches_are_noops(gpu):
    """Zero groups / zero packets: every entry point returns OK and touches nothing
    (upstream Encode/Reconstruct on an empty batch is never reached by ugo, but
    a batch API must accept it)."""
    enc = fec.New(10, 3)
    for shard_major in (False, True):
        shape = (13, 0, 1360) if shard_major else (0, 13, 1360)
        t = torch.empty(shape, dtype=torch.uint8, device="cuda")
        enc.encode_batch(t, shard_size=1350, shard_major=shard_major)
        enc.reconstruct_batch(t, torch.empty(0, dtype=torch.int64, device="cuda"), shard_size=1350,
                              shard_major=shard_major)
    host = np.empty((0, 13, 1360), np.uint8)
    enc.encode_host(host, 1350)
    assert enc.reconstruct_host(host, np.empty(0, np.uint64), 1350) == 0
    sh = torch.zeros((13, 4, 1472), dtype=torch.uint8, device="cuda")
    present = torch.zeros(4, dtype=torch.int64, device="cuda")
    enc.rx_assemble(torch.empty((0, 1488), dtype=torch.uint8, device="cuda"),
                    torch.empty(0, dtype=torch.int16, device="cuda"), sh, present, shard_size=1470)
    assert not present.any() and not sh.any()
    enc.tx_assemble(torch.empty((0, 1488), dtype=torch.uint8, device="cuda"),
                    torch.empty(0, dtype=torch.int16, device="cuda"),
                    torch.empty((0, 1488), dtype=torch.uint8, device="cuda"),
                    torch.empty(0, dtype=torch.int16, device="cuda"))
    torch.cuda.synchronize()


def _wide_masks(G, n, p, rng):
    """[G][W] presence words (W = ceil(n/64)) with 0..p+1 erasures per group
    (p+1: a too-few-shards group), plus the per-group erased-row sets."""
    W = (n + 63) // 64
    words = np.zeros((G, W), np.uint64)
    erased = []
    for g in range(G):
        e = int(rng.integers(0, p + 2)) if g else p  # group 0: as many erasures as recoverable
        er = set(int(r) for r in rng.choice(n, size=min(e, n), replace=False))
        erased.append(er)
        for r in range(n):
            if r not in er:
                words[g, r >> 6] |= np.uint64(1 << (r & 63))
    return words, erased


@pytest.mark.parametrize("d,p,S,G", [(70, 10, 40, 6),    # d > 32: byte kernel, descriptors built on the host
                                     (60, 8, 1104, 4),   # d > 32, 69 chunks: streaming k_apply_q
                                     (72, 20, 160, 3),   # d > 32, p > 8, 10 chunks: k_apply_qa in passes
                                     (30, 40, 48, 5),    # d <= 32, p > 8: k_apply
                                     (8, 248, 16, 3)])   # 256 shards, upstream's maximum
def test_more_than_64_shards(gpu, d, p, S, G):
    """Upstream allows 256 shards: encode, batch reconstruct (in place and into
    separate outputs, W = ceil((d+p)/64) presence words per group) and the
    per-group Reconstruct against the independent Python restatement
    (oracle/rs_ref.py reconstruct_group: first d present rows, two-stage)."""
    n = d + p
    host = _rand(G, n, S, 7 + n).numpy()
    want = host.copy()
    rs_ref.c_encode(d, p, want, S=S)
    enc = fec.New(d, p)
    assert enc.mask_words == (n + 63) // 64
    t = _dev(host)
    enc.encode_batch(t, shard_size=S)
    assert np.array_equal(t.cpu().numpy(), want)
    M = rs_ref.build_matrix(d, p)
    words, erased = _wide_masks(G, n, p, np.random.default_rng(n))
    exp, exp_st = [], []
    for g in range(G):
        rows = [None if r in erased[g] else bytearray(want[g, r].tobytes()) for r in range(n)]
        err = rs_ref.reconstruct_group(M, d, p, rows)
        exp_st.append(0 if err is None else fec.ErrTooFewShards.code)
        exp.append(rows)
    inp = want.copy()
    for g in range(G):
        for r in erased[g]:
            inp[g, r] = 0
    dm = torch.as_tensor(words.view(np.int64)).cuda()
    # in place
    t = _dev(inp)
    st = torch.full((G,), -1, dtype=torch.int8, device="cuda")
    enc.reconstruct_batch(t, dm, shard_size=S, status=st)
    got, got_st = t.cpu().numpy(), st.cpu().numpy()
    assert list(got_st) == exp_st
    for g in range(G):
        for r in range(n):
            if exp_st[g] == 0:
                assert got[g, r].tobytes() == bytes(exp[g][r]), (g, r)
            else:
                assert np.array_equal(got[g, r], inp[g, r]), (g, r)  # too few shards: untouched
    # into separate outputs (slot i = i-th erased row)
    out = torch.full((G, p, S), 0xA5, dtype=torch.uint8, device="cuda")
    enc.reconstruct_into(_dev(inp), dm, out, shard_size=S, out_shard_major=False)
    o = out.cpu().numpy()
    for g in range(G):
        if exp_st[g] == 0:
            for i, r in enumerate(sorted(erased[g])):
                assert o[g, i].tobytes() == bytes(exp[g][r]), (g, i)
    # host batch (pinned zero-copy path) and the Go-shaped per-group call
    hb = fec.host_alloc(G * n * S).reshape(G, n, S)
    hb[:] = inp
    hst = np.full(G, -1, np.int8)
    enc.reconstruct_host(hb, words, S, status=hst)
    assert list(hst) == exp_st
    assert np.array_equal(hb, got)
    fec.host_free(hb)
    g = 0
    shards = [None if r in erased[g] else bytearray(want[g, r].tobytes()) for r in range(n)]
    enc.Reconstruct(shards)
    assert [bytes(x) for x in shards] == [bytes(x) for x in exp[g]]


@pytest.mark.parametrize("d,p,S,pitch,opitch,shard_major,table_max",
                         [(10, 3, 1350, 1360, 1360, True, "16"),    # headline kernel (k_apply_p)
                          (10, 3, 1350, 1360, 1360, False, "0"),    # k_prepare + per-group descriptors
                          (32, 8, 9000, 9008, 9008, True, "16"),    # jumbo: wave-aligned groups (k_apply_qa)
                          (32, 8, 1000, 1008, 1024, False, "16"),   # 63 chunks: k_apply_qa, 1 idle lane per group
                          (10, 6, 1008, 1008, 1008, True, "16"),    # MODE 1 table, p > 4: k_apply_qa
                          (20, 4, 2000, 2000, 2016, False, "16"),   # MODE 2, e <= 4: k_apply_qa<4>
                          (16, 4, 1030, 1040, 1040, True, "16"),    # 65 chunks: streaming k_apply_q
                          (10, 3, 1350, 1353, 1355, False, "16"),   # unaligned: byte kernel
                          (6, 2, 77, 80, 96, True, "16"),           # rows < 64 chunks: k_apply
                          (12, 4, 1030, 1040, 1040, False, "16"),   # p = 4
                          (20, 9, 1100, 1104, 1104, True, "16")])   # p > 8 (k_prepare + k_apply)
def test_reconstruct_into_vs_oracle(gpu, d, p, S, pitch, opitch, shard_major, table_max, monkeypatch):
    """ugo_fec_reconstruct_into: shards only read; output i = i-th erased row
    (ascending), bit-exact vs the oracle's in-place result; slots past e and
    failing groups untouched; statuses as the in-place form."""
    monkeypatch.setenv("UGO_FEC_TABLE_MAX_SHARDS", table_max)
    n, G = d + p, 700
    host = _rand(G, n, pitch, 77 + d + p).numpy()
    rs_ref.c_encode(d, p, host, S=S)
    rng = np.random.default_rng(d * 7 + p)
    masks = np.zeros(G, np.uint64)
    for g in range(G):
        e = int(rng.integers(0, p + 2))  # includes e = 0 and too-few-shards groups
        m = (1 << n) - 1
        for r in rng.choice(n, size=min(e, n), replace=False):
            m &= ~(1 << int(r))
        masks[g] = m
    inp = _erase(host, masks, n)
    inp[:, :, S:] = 0x3C  # padding stays what it was in the input
    enc = fec.New(d, p)
    for data_only in (False, True):
        want = inp.copy()
        rc, want_st = rs_ref.c_reconstruct(d, p, want, masks, S=S, data_only=data_only)
        exp = np.full((G, p, opitch), 0xA5, dtype=np.uint8)
        for g in range(G):
            if want_st[g] != 0:
                continue
            er = [r for r in range(n) if not (int(masks[g]) >> r) & 1 and (r < d or not data_only)]
            for i, r in enumerate(er):
                exp[g, i, :S] = want[g, r, :S]
        t_in = _dev(np.ascontiguousarray(inp.transpose(1, 0, 2)) if shard_major else inp)
        before = t_in.clone()
        out = torch.full((p, G, opitch) if shard_major else (G, p, opitch), 0xA5, dtype=torch.uint8, device="cuda")
        st = torch.full((G,), -1, dtype=torch.int8, device="cuda")
        enc.reconstruct_into(t_in, _masks_to_dev(masks), out, shard_size=S, data_only=data_only, status=st,
                             shard_major=shard_major, out_shard_major=shard_major)
        torch.cuda.synchronize()
        assert torch.equal(t_in, before), "reconstruct_into wrote its input"
        assert np.array_equal(st.cpu().numpy(), want_st)
        got = out.cpu().numpy()
        if shard_major:
            got = got.transpose(1, 0, 2)
        assert np.array_equal(got, exp), (d, p, S, data_only)


@pytest.mark.parametrize("d,p,S,pitch,shard_major,G", [
    (10, 3, 1470, 1472, True, 900),   # ugo's RX batch: k_apply_p list form, wave spans 2 list entries
    (10, 3, 1350, 1360, False, 333),  # group-major
    (6, 2, 77, 80, True, 257),        # rows < 64 chunks: k_apply list form
    (12, 4, 1030, 1040, True, 100),   # p = 4
    (10, 5, 1200, 1200, False, 64),   # p > 4 (epad 8): k_apply list form
    (10, 3, 1470, 1472, True, 1),     # one group
])
def test_lossy_list_and_reconstruct_list_vs_oracle(gpu, d, p, S, pitch, shard_major, G):
    """ugo_fec_lossy_groups lists exactly the groups with an erased (data) row,
    ascending; ugo_fec_reconstruct_list then matches the oracle's Reconstruct
    for list entry j: outputs compact in list order (or in place), status[j];
    entries past the count and the input batch untouched."""
    n = d + p
    host = _rand(G, n, pitch, 91 + d + p + G).numpy()
    rs_ref.c_encode(d, p, host, S=S)
    rng = np.random.default_rng(G + d)
    masks = np.zeros(G, np.uint64)
    for g in range(G):
        e = int(rng.choice([0, 0, 1, 2, p, p + 1]))  # complete, lossy and too-few-shards groups
        m = (1 << n) - 1
        for r in rng.choice(n, size=min(e, n), replace=False):
            m &= ~(1 << int(r))
        masks[g] = m
    inp = _erase(host, masks, n)
    enc = fec.New(d, p)
    dm = _masks_to_dev(masks)
    t_in = _dev(np.ascontiguousarray(inp.transpose(1, 0, 2)) if shard_major else inp)
    for data_only in (True, False):
        scope = ((1 << d) - 1) if data_only else ((1 << n) - 1)
        want_list = [g for g in range(G) if (~int(masks[g])) & scope]
        lst, cnt = enc.lossy_groups(dm, data_only=data_only)
        k = int(cnt.item())
        assert lst.cpu().numpy()[:k].tolist() == want_list
        want = inp.copy()
        rc, want_st = rs_ref.c_reconstruct(d, p, want, masks, S=S, data_only=data_only)
        slots = min(d, p) if data_only else p
        out = torch.full((G, slots, pitch), 0xA5, dtype=torch.uint8, device="cuda")
        st = torch.full((G,), -1, dtype=torch.int8, device="cuda")
        before = t_in.clone()
        enc.reconstruct_list(t_in, dm, lst, cnt, out, shard_size=S, data_only=data_only, status=st,
                             shard_major=shard_major)
        torch.cuda.synchronize()
        assert torch.equal(t_in, before), "reconstruct_list wrote its input"
        o, s_ = out.cpu().numpy(), st.cpu().numpy()
        exp = np.full_like(o, 0xA5)
        for j, g in enumerate(want_list):
            assert s_[j] == want_st[g], (j, g)
            if want_st[g] != 0:
                continue
            er = [r for r in range(n) if not (int(masks[g]) >> r) & 1 and (r < d or not data_only)]
            for i, r in enumerate(er):
                exp[j, i, :S] = want[g, r, :S]
        assert np.array_equal(o, exp), (d, p, S, data_only)
        assert (s_[k:] == -1).all()
        # in place: the erased rows of the listed groups rebuilt in the batch itself
        t_ip = t_in.clone()
        enc.reconstruct_list(t_ip, dm, lst, cnt, None, shard_size=S, data_only=data_only, shard_major=shard_major)
        got = t_ip.cpu().numpy()
        if shard_major:
            got = got.transpose(1, 0, 2)
        exp_ip = inp.copy()
        for g in want_list:
            if want_st[g] == 0:
                for r in range(n):
                    if not (int(masks[g]) >> r) & 1 and (r < d or not data_only):
                        exp_ip[g, r, :S] = want[g, r, :S]
        assert np.array_equal(got, exp_ip)


@pytest.mark.parametrize("G", [4096, 4097, 70000, 4 * 1048576 + 123])
def test_lossy_list_many_tiles(gpu, G):
    """The one-launch lossy list (k_lossy_list1: each 4,096-group tile publishes
    its counts, every tile sums the tiles before it) over 1 to 1,025 tiles,
    against numpy: the list, its count, and -- through ugo_fec_recover_data --
    each entry's row offset (the recovered rows' places, in `recovered` order).
    Repeated calls on two streams alternate, so each stream's count words are
    reused with new epochs; a tile whose groups are all complete publishes 0."""
    d, p = 10, 3
    n = d + p
    rng = np.random.default_rng(G)
    full = (1 << n) - 1
    masks = np.full(G, full, np.uint64)
    lossy = rng.random(G) < 0.3
    lossy[G // 3: G // 3 + 9000] = False  # whole complete tiles in the middle
    for k in range(1, 5):  # 1..4 erased rows, some below d shards
        sel = lossy & (rng.integers(1, 5, G) == k)
        for _ in range(k):
            masks[sel] &= ~(np.uint64(1) << rng.integers(0, n, G).astype(np.uint64))[sel]
    dm = _masks_to_dev(masks)
    torch.cuda.synchronize()  # the masks are on the default stream; the calls below run on two others
    enc = fec.New(d, p)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    lst = torch.empty(G, dtype=torch.int32, device="cuda")
    for data_only in (True, False, True):
        scope = np.uint64(((1 << d) - 1) if data_only else full)
        want = np.nonzero((~masks) & np.uint64(full) & scope)[0]
        for call in range(3):
            s = streams[call % 2]
            with torch.cuda.stream(s):
                lst.fill_(-1)
                _, cnt = enc.lossy_groups(dm, data_only=data_only, out=lst, stream=s)
            s.synchronize()
            k = int(cnt.item())
            assert k == len(want), (data_only, call)
            assert np.array_equal(lst[:k].cpu().numpy(), want.astype(np.int32)), (data_only, call)
            assert (lst[k:] == -1).all()
    if G > 100000:
        return
    # row offsets: the places ugo_fec_recover_data writes for each recovered row
    S, pitch = 16, 16
    sh = torch.zeros((n, G, pitch), dtype=torch.uint8, device="cuda")
    have = np.zeros(G, np.int64)
    for r in range(n):
        have += ((masks >> np.uint64(r)) & np.uint64(1)).astype(np.int64)
    want_idx = [g * n + r for g in np.nonzero(have >= d)[0] for r in range(d) if not (int(masks[g]) >> r) & 1]
    out = torch.empty((len(want_idx), pitch), dtype=torch.uint8, device="cuda")
    idx = torch.full((len(want_idx),), -1, dtype=torch.int32, device="cuda")
    cnt = enc.recover_data(sh, dm, out, idx, shard_size=S)
    assert int(cnt.item()) == len(want_idx)
    assert idx.cpu().numpy().tolist() == want_idx


@pytest.mark.parametrize("d,p,S,pitch,shard_major,G", [
    (10, 3, 1470, 1472, True, 900),   # ugo's RX batch: k_apply_p list form
    (10, 3, 1350, 1360, False, 333),  # group-major
    (6, 2, 77, 80, True, 257),        # rows < 64 chunks: k_apply list form
    (10, 5, 1200, 1200, False, 64),   # p > 4: k_apply list form
])
def test_recover_data_vs_oracle(gpu, d, p, S, pitch, shard_major, G):
    """ugo_fec_recover_data: `input`'s recovered list of a device batch (groups
    ascending, lost data rows ascending, groups below d shards nothing) against
    the oracle's ReconstructData, row-compact with each shard's place; the
    count on the device; max_rows below the count writes only that many rows."""
    n = d + p
    host = _rand(G, n, pitch, 93 + d + p + G).numpy()
    rs_ref.c_encode(d, p, host, S=S)
    rng = np.random.default_rng(G + d + 7)
    masks = np.zeros(G, np.uint64)
    for g in range(G):
        e = int(rng.choice([0, 0, 1, 2, p, p + 1]))
        m = (1 << n) - 1
        for r in rng.choice(n, size=min(e, n), replace=False):
            m &= ~(1 << int(r))
        masks[g] = m
    inp = _erase(host, masks, n)
    enc = fec.New(d, p)
    dm = _masks_to_dev(masks)
    t_in = _dev(np.ascontiguousarray(inp.transpose(1, 0, 2)) if shard_major else inp)
    want = inp.copy()
    rc, want_st = rs_ref.c_reconstruct(d, p, want, masks, S=S, data_only=True)
    rec = [(g, r) for g in range(G) if want_st[g] == 0 for r in range(d) if not (int(masks[g]) >> r) & 1]
    opitch = (S + 15) // 16 * 16
    for max_rows in (max(len(rec), 1), max(len(rec) // 2, 1)):
        out = torch.full((max_rows, opitch), 0xA5, dtype=torch.uint8, device="cuda")
        idx = torch.full((max_rows,), -1, dtype=torch.int32, device="cuda")
        before = t_in.clone()
        cnt = enc.recover_data(t_in, dm, out, idx, shard_size=S, shard_major=shard_major)
        torch.cuda.synchronize()
        assert torch.equal(t_in, before), "recover_data wrote its input"
        assert int(cnt.item()) == len(rec)
        m = min(max_rows, len(rec))
        o, ix = out.cpu().numpy(), idx.cpu().numpy()
        assert ix[:m].tolist() == [g * n + r for g, r in rec[:m]]
        assert (ix[m:] == -1).all()
        for k, (g, r) in enumerate(rec[:m]):
            assert np.array_equal(o[k, :S], want[g, r, :S]), (k, g, r)
        assert (o[m:] == 0xA5).all()


@pytest.mark.parametrize("d,p,S,G,table_max", [
    (10, 3, 1350, 777, "16"),   # the bench's dense rows: 8 groups per pseudo-group, k_apply_p on 2-B aligned groups
    (10, 3, 1350, 777, "0"),    # same with per-group descriptors (k_prepare)
    (10, 3, 1476, 64, "16"),    # ugo's full packet size: 4 groups per pseudo-group
    (12, 4, 1031, 333, "16"),   # odd S: 16 groups per pseudo-group, 1-B aligned groups
    (4, 2, 1009, 100, "16"),    # exactly 64 chunks per row
    (10, 3, 1350, 7, "16"),     # fewer groups than one pseudo-group: the tail alone
    (10, 3, 1350, 1, "16"),     # one group
    (20, 4, 1350, 99, "16"),    # d > 16: dense encode, byte-kernel reconstruct
    (10, 3, 100, 50, "16"),     # rows < 64 chunks: dense encode, byte-kernel reconstruct
])
def test_dense_planar_rows_vs_oracle(gpu, d, p, S, G, table_max, monkeypatch):
    """Dense shard-major batches (group stride == S, rows 16-B aligned: no
    padding bytes at all): encode folds 16/gcd(S,16) groups into one
    pseudo-group, reconstruct runs the vector kernel on unaligned group
    offsets.  Bit-exact vs the oracle in place and into a dense output batch;
    the bytes between rows are never written."""
    monkeypatch.setenv("UGO_FEC_TABLE_MAX_SHARDS", table_max)
    n = d + p
    rs = (G * S + 15) // 16 * 16 + 32
    rng = np.random.default_rng(S * 31 + G)
    packed = rng.integers(0, 256, (G, n, S), dtype=np.uint8)
    want = packed.copy()
    rs_ref.c_encode(d, p, want, S=S)
    flat = torch.full((n * rs,), 0x5A, dtype=torch.uint8, device="cuda")
    view = flat.as_strided((n, G, S), (rs, S, 1))
    view.copy_(torch.as_tensor(packed).cuda().transpose(0, 1))
    outside = torch.ones(n * rs, dtype=torch.bool, device="cuda")
    outside.as_strided((n, G, S), (rs, S, 1)).fill_(False)
    untouched = flat.clone()
    enc = fec.New(d, p)
    enc.encode_batch(view, shard_size=S, shard_major=True)
    assert np.array_equal(view.transpose(0, 1).cpu().numpy(), want)
    assert torch.equal(flat[outside], untouched[outside]), "bytes between rows were written"
    masks = np.zeros(G, np.uint64)
    for g in range(G):
        m = (1 << n) - 1
        for r in rng.choice(n, size=int(rng.integers(0, p + 2)), replace=False):
            m &= ~(1 << int(r))
        masks[g] = m
    inp = _erase(want, masks, n)
    exp = inp.copy()
    rc, exp_st = rs_ref.c_reconstruct(d, p, exp, masks, S=S)
    # into a dense, contiguous [p][G][S] output batch (its rows need no alignment)
    out = torch.full((p, G, S), 0xA5, dtype=torch.uint8, device="cuda")
    view.copy_(torch.as_tensor(inp).cuda().transpose(0, 1))
    st = torch.full((G,), -1, dtype=torch.int8, device="cuda")
    enc.reconstruct_into(view, _masks_to_dev(masks), out, shard_size=S, status=st, shard_major=True,
                         out_shard_major=True)
    torch.cuda.synchronize()
    assert np.array_equal(st.cpu().numpy(), exp_st)
    o = out.transpose(0, 1).cpu().numpy()
    want_o = np.full((G, p, S), 0xA5, dtype=np.uint8)
    for g in range(G):
        if exp_st[g] != 0:
            continue
        for i, r in enumerate([r for r in range(n) if not (int(masks[g]) >> r) & 1]):
            want_o[g, i] = exp[g, r]
    assert np.array_equal(o, want_o)
    # in place
    st.fill_(-1)
    enc.reconstruct_batch(view, _masks_to_dev(masks), shard_size=S, status=st, shard_major=True)
    assert np.array_equal(st.cpu().numpy(), exp_st)
    assert np.array_equal(view.transpose(0, 1).cpu().numpy(), exp)
    assert torch.equal(flat[outside], untouched[outside])


@settings(max_examples=int(os.environ.get("UGO_HYP_EXAMPLES", "150")) // 5, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(d=st.integers(1, 16), p=st.integers(1, 4), S=st.integers(900, 2100), G=st.integers(1, 160),
       table=st.sampled_from(["16", "0"]), seed=st.integers(0, 2**31 - 1))
def test_random_dense_rows_vs_oracle(gpu, d, p, S, G, table, seed, monkeypatch):
    """Random dense shard-major batches around the k_apply_pd threshold
    (S >= 1009) and every pseudo-group fold (any S mod 16): encode, reconstruct
    in place and into a dense output batch, bit-exact vs the oracle."""
    monkeypatch.setenv("UGO_FEC_TABLE_MAX_SHARDS", table)
    n = d + p
    rs = (G * S + 15) // 16 * 16
    rng = np.random.default_rng(seed)
    packed = rng.integers(0, 256, (G, n, S), dtype=np.uint8)
    want = packed.copy()
    rs_ref.c_encode(d, p, want, S=S)
    flat = torch.zeros((n * rs,), dtype=torch.uint8, device="cuda")
    view = flat.as_strided((n, G, S), (rs, S, 1))
    view.copy_(torch.as_tensor(packed).cuda().transpose(0, 1))
    enc = fec.New(d, p)
    enc.encode_batch(view, shard_size=S, shard_major=True)
    assert np.array_equal(view.transpose(0, 1).cpu().numpy(), want)
    masks = np.zeros(G, np.uint64)
    for g in range(G):
        m = (1 << n) - 1
        for r in rng.choice(n, size=int(rng.integers(0, p + 2)), replace=False):
            m &= ~(1 << int(r))
        masks[g] = m
    inp = _erase(want, masks, n)
    exp = inp.copy()
    rc, exp_st = rs_ref.c_reconstruct(d, p, exp, masks, S=S)
    view.copy_(torch.as_tensor(inp).cuda().transpose(0, 1))
    out = torch.full((p, G, S), 0xA5, dtype=torch.uint8, device="cuda")
    st = torch.full((G,), -1, dtype=torch.int8, device="cuda")
    enc.reconstruct_into(view, _masks_to_dev(masks), out, shard_size=S, status=st, shard_major=True,
                         out_shard_major=True)
    assert np.array_equal(st.cpu().numpy(), exp_st)
    o = out.transpose(0, 1).cpu().numpy()
    for g in range(G):
        er = [r for r in range(n) if not (int(masks[g]) >> r) & 1] if exp_st[g] == 0 else []
        for i in range(p):
            assert np.array_equal(o[g, i], exp[g, er[i]] if i < len(er) else np.full(S, 0xA5, np.uint8)), (g, i)
    enc.reconstruct_batch(view, _masks_to_dev(masks), shard_size=S, shard_major=True)
    assert np.array_equal(view.transpose(0, 1).cpu().numpy(), exp)


def test_reconstruct_into_rejects_bad_outputs(gpu):
    d, p, S = 10, 3, 1350
    enc = fec.New(d, p)
    lib = fec.load_library()
    t = torch.zeros((4, d + p, 1360), dtype=torch.uint8, device="cuda")
    m = _masks_to_dev(np.full(4, (1 << (d + p)) - 2, np.uint64))
    o = torch.zeros((4, p, 1360), dtype=torch.uint8, device="cuda")
    pitch = 1360
    args = (enc._h, t.data_ptr(), m.data_ptr(), 4, S, pitch, (d + p) * pitch)
    assert lib.ugo_fec_reconstruct_into(*args, None, pitch, p * pitch, 0, None, None) == fec.ErrInvalidArg.code
    assert lib.ugo_fec_reconstruct_into(*args, o.data_ptr(), S - 1, p * pitch, 0, None, None) == fec.ErrInvalidArg.code
    assert lib.ugo_fec_reconstruct_into(*args, o.data_ptr(), pitch, S - 1, 0, None, None) == fec.ErrInvalidArg.code
    assert lib.ugo_fec_reconstruct_into(*args, o.data_ptr(), pitch, p * pitch, 0, None, None) == 0
    torch.cuda.synchronize()
    assert torch.equal(o[:, 0, :S], torch.zeros_like(o[:, 0, :S]))  # all-zero codeword: row 0 rebuilt as zeros


def test_overlapping_batch_layouts_rejected(gpu):
    """Strided batches whose shard slots overlap (kernels would write rows
    other lanes read) are refused before any launch; the disjoint group-major
    and planar layouts of the same buffer are accepted."""
    d, p, S, G = 10, 3, 1350, 4
    n, pitch = d + p, 1360
    enc = fec.New(d, p)
    lib = fec.load_library()
    t = torch.zeros((G * n + 2, pitch), dtype=torch.uint8, device="cuda")
    m = _masks_to_dev(np.full(G, (1 << n) - 2, np.uint64))
    bad = [(pitch, (n - 1) * pitch),       # group g's last row is group g+1's first
           (2 * pitch, pitch),             # groups interleave into each other's rows
           (S - 1, n * pitch)]             # rows overlap inside a group
    good = [(pitch, n * pitch), (G * pitch, pitch)]
    for rs, gs in bad:
        assert lib.ugo_fec_encode_strided(enc._h, t.data_ptr(), G, S, rs, gs, None) == fec.ErrInvalidArg.code
        assert lib.ugo_fec_reconstruct_strided(enc._h, t.data_ptr(), m.data_ptr(), G, S, rs, gs, 0, None,
                                               None) == fec.ErrInvalidArg.code
    for rs, gs in good:
        assert lib.ugo_fec_encode_strided(enc._h, t.data_ptr(), G, S, rs, gs, None) == 0
        assert lib.ugo_fec_reconstruct_strided(enc._h, t.data_ptr(), m.data_ptr(), G, S, rs, gs, 0, None, None) == 0
    torch.cuda.synchronize()
    assert not bool(t.any())  # all-zero codewords stay zero
    # the binding's size checks are explicit (they hold under python -O)
    with pytest.raises(ValueError):
        enc.reconstruct_batch(t[: G * n].view(G, n, pitch), m[:-1], shard_size=S)
    with pytest.raises(ValueError):
        enc.reconstruct_into(t[: G * n].view(G, n, pitch), m, torch.zeros((p, G - 1, pitch), dtype=torch.uint8,
                                                                          device="cuda"), shard_size=S)


@settings(max_examples=int(os.environ.get("UGO_HYP_EXAMPLES", "150")), deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(d=st.integers(1, 48), p=st.integers(1, 16), S=st.integers(1, 2100), pad=st.sampled_from([0, 3, 16]),
       table=st.sampled_from(["16", "0"]), seed=st.integers(0, 2**31 - 1))
def test_random_geometries_vs_oracle(gpu, d, p, S, pad, table, seed, monkeypatch):
    """Random codes, shard sizes and pitches (aligned and not, so every launch
    path -- perm tables, streaming, wave-aligned, passes, masked Horner, byte
    kernel; table and per-group descriptors -- gets drawn): encode and
    reconstruct (in place, data-only, into) bit-exact vs the C oracle."""
    n = d + p
    if n > 64:
        return
    monkeypatch.setenv("UGO_FEC_TABLE_MAX_SHARDS", table)
    pitch = S + pad
    G = 48
    rng = np.random.default_rng(seed)
    host = rng.integers(0, 256, (G, n, pitch), dtype=np.uint8)
    want = host.copy()
    rs_ref.c_encode(d, p, want, S=S)
    enc = fec.New(d, p)
    t = _dev(host)
    enc.encode_batch(t, shard_size=S)
    assert np.array_equal(t.cpu().numpy()[:, :, :S], want[:, :, :S])
    masks = np.zeros(G, np.uint64)
    for g in range(G):
        e = int(rng.integers(0, p + 2))
        m = (1 << n) - 1
        for r in rng.choice(n, size=min(e, n), replace=False):
            m &= ~(1 << int(r))
        masks[g] = m
    inp = _erase(want, masks, n)
    for data_only in (False, True):
        exp = inp.copy()
        rc, exp_st = rs_ref.c_reconstruct(d, p, exp, masks, S=S, data_only=data_only)
        t = _dev(inp)
        stt = torch.full((G,), -1, dtype=torch.int8, device="cuda")
        enc.reconstruct_batch(t, _masks_to_dev(masks), shard_size=S, data_only=data_only, status=stt)
        assert np.array_equal(stt.cpu().numpy(), exp_st)
        assert np.array_equal(t.cpu().numpy()[:, :, :S], exp[:, :, :S]), (d, p, S, pitch, data_only)
    out = torch.full((G, p, pitch), 0xA5, dtype=torch.uint8, device="cuda")
    enc.reconstruct_into(_dev(inp), _masks_to_dev(masks), out, shard_size=S, out_shard_major=False)
    o = out.cpu().numpy()
    exp = inp.copy()
    rc, exp_st = rs_ref.c_reconstruct(d, p, exp, masks, S=S)
    for g in range(G):
        if exp_st[g] != 0:
            continue
        er = [r for r in range(n) if not (int(masks[g]) >> r) & 1]
        for i, r in enumerate(er):
            assert np.array_equal(o[g, i, :S], exp[g, r, :S]), (d, p, S, pitch, g, i)


@settings(max_examples=int(os.environ.get("UGO_HYP_EXAMPLES", "150")) // 3, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(d=st.integers(1, 24), p=st.integers(1, 8), S=st.integers(1, 1500), planar=st.booleans(),
       row_pad=st.sampled_from([0, 16, 48, 4096]), group_pad=st.sampled_from([0, 3, 16, 112]),
       seed=st.integers(0, 2**31 - 1))
def test_random_strided_layouts_vs_oracle(gpu, d, p, S, planar, row_pad, group_pad, seed):
    """Strided batch views (the tensor's own row and group strides, padded
    either way, group-major or planar) encode and reconstruct like the packed
    batch, and bytes outside the shards are never written."""
    n, G = d + p, 40
    pitch = (S + 15) // 16 * 16
    rng = np.random.default_rng(seed)
    packed = rng.integers(0, 256, (G, n, pitch), dtype=np.uint8)
    want = packed.copy()
    rs_ref.c_encode(d, p, want, S=S)
    if planar:
        rs, gs = G * pitch + row_pad, pitch + group_pad
        if group_pad:
            rs = G * gs + row_pad
        shape, strides = (n, G, pitch), (rs, gs, 1)
        total = (n - 1) * rs + (G - 1) * gs + pitch
    else:
        rs, gs = pitch + row_pad, n * (pitch + row_pad) + group_pad
        shape, strides = (G, n, pitch), (gs, rs, 1)
        total = (G - 1) * gs + (n - 1) * rs + pitch
    flat = torch.full((total,), 0x5A, dtype=torch.uint8, device="cuda")
    view = flat.as_strided(shape, strides)
    src = torch.as_tensor(packed).cuda()
    view.copy_(src.transpose(0, 1) if planar else src)
    untouched = flat.clone()
    mask_out = torch.ones(total, dtype=torch.bool, device="cuda")
    mask_out.as_strided(shape, strides)[..., :S] = False  # shard bytes
    enc = fec.New(d, p)
    enc.encode_batch(view, shard_size=S, shard_major=planar)
    got = (view.transpose(0, 1) if planar else view).cpu().numpy()
    assert np.array_equal(got[:, :, :S], want[:, :, :S])
    assert torch.equal(flat[mask_out], untouched[mask_out]), "bytes outside the shards were written"
    masks = np.zeros(G, np.uint64)
    for g in range(G):
        m = (1 << n) - 1
        for r in rng.choice(n, size=int(rng.integers(0, p + 1)), replace=False):
            m &= ~(1 << int(r))
        masks[g] = m
    inp = _erase(want, masks, n)
    view.copy_(torch.as_tensor(inp).cuda().transpose(0, 1) if planar else torch.as_tensor(inp).cuda())
    enc.reconstruct_batch(view, _masks_to_dev(masks), shard_size=S, shard_major=planar)
    got = (view.transpose(0, 1) if planar else view).cpu().numpy()
    assert np.array_equal(got[:, :, :S], want[:, :, :S])


@settings(max_examples=int(os.environ.get("UGO_HYP_EXAMPLES", "150")) // 5, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(d=st.integers(1, 40), p=st.integers(1, 12), S=st.integers(1, 1500), pad=st.sampled_from([0, 5, 16]),
       G=st.integers(1, 200), pinned=st.booleans(), data_only=st.booleans(), seed=st.integers(0, 2**31 - 1))
def test_random_host_batches_vs_oracle(gpu, d, p, S, pad, G, pinned, data_only, seed):
    """The host-memory entry points (staged DMA for pageable batches, zero-copy
    for pinned ones) on random codes and sizes: encode and reconstruct
    (statuses included) bit-exact vs the oracle."""
    n = d + p
    if n > 64:
        return
    pitch = S + pad
    rng = np.random.default_rng(seed)
    host = rng.integers(0, 256, (G, n, pitch), dtype=np.uint8)
    want = host.copy()
    rs_ref.c_encode(d, p, want, S=S)
    enc = fec.New(d, p)
    if pinned:
        buf = fec.host_alloc(G * n * pitch).reshape(G, n, pitch)
    else:
        buf = np.empty((G, n, pitch), np.uint8)
    try:
        buf[:] = host
        enc.encode_host(buf, S)
        assert np.array_equal(buf[:, :, :S], want[:, :, :S])
        masks = np.zeros(G, np.uint64)
        for g in range(G):
            m = (1 << n) - 1
            for r in rng.choice(n, size=min(int(rng.integers(0, p + 2)), n), replace=False):
                m &= ~(1 << int(r))
            masks[g] = m
        inp = _erase(want, masks, n)
        exp = inp.copy()
        rc, exp_st = rs_ref.c_reconstruct(d, p, exp, masks, S=S, data_only=data_only)
        buf[:] = inp
        stt = np.full(G, -1, np.int8)
        enc.reconstruct_host(buf, masks, S, data_only=data_only, status=stt)
        assert np.array_equal(stt, exp_st)
        assert np.array_equal(buf[:, :, :S], exp[:, :, :S])
    finally:
        if pinned:
            fec.host_free(buf)


@pytest.mark.parametrize("d,p,S,pitch", [(10, 3, 1_000_003, 1_000_016),   # 62,501 chunks per row
                                         (32, 8, 262_144, 262_144),       # jumbo code, 256-KiB shards
                                         (10, 3, 70_000, 70_003)])        # > 64 KiB, unaligned: byte kernel
def test_large_shards_vs_oracle(gpu, d, p, S, pitch):
    """Shards far past ugo's 1,476 B (sizes are size_t in the ABI): encode and
    every recoverable erasure count, bit-exact vs the oracle."""
    n, G = d + p, 4
    host = _rand(G, n, pitch, S % 1000).numpy()
    want = host.copy()
    rs_ref.c_encode(d, p, want, S=S)
    enc = fec.New(d, p)
    t = _dev(host)
    enc.encode_batch(t, shard_size=S)
    assert np.array_equal(t.cpu().numpy()[:, :, :S], want[:, :, :S])
    rng = np.random.default_rng(S)
    masks = np.zeros(G, np.uint64)
    for g in range(G):
        m = (1 << n) - 1
        for r in rng.choice(n, size=g * p // (G - 1), replace=False):  # 0 .. p erasures
            m &= ~(1 << int(r))
        masks[g] = m
    inp = _erase(want, masks, n)
    t = _dev(inp)
    enc.reconstruct_batch(t, _masks_to_dev(masks), shard_size=S)
    assert np.array_equal(t.cpu().numpy()[:, :, :S], want[:, :, :S])


@settings(max_examples=int(os.environ.get("UGO_HYP_EXAMPLES", "150")) // 10, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])
@given(d=st.integers(1, 16), p=st.integers(49, 120), S=st.integers(1, 48), pad=st.sampled_from([0, 16]),
       seed=st.integers(0, 2**31 - 1))
def test_random_wide_codes_vs_restatement(gpu, d, p, S, pad, seed):
    """Random codes past 64 shards (multi-word presence masks, host-built
    descriptors): encode vs the C oracle, reconstruct (in place) vs the
    independent Python restatement, aligned and unaligned pitches."""
    n = d + p
    pitch = (S + 15) // 16 * 16 + pad if pad else S
    G = 3
    rng = np.random.default_rng(seed)
    host = rng.integers(0, 256, (G, n, pitch), dtype=np.uint8)
    want = host.copy()
    rs_ref.c_encode(d, p, want, S=S)
    enc = fec.New(d, p)
    t = _dev(host)
    enc.encode_batch(t, shard_size=S)
    assert np.array_equal(t.cpu().numpy()[:, :, :S], want[:, :, :S])
    M = rs_ref.build_matrix(d, p)
    words, erased = _wide_masks(G, n, p, rng)
    inp = want.copy()
    for g in range(G):
        for r in erased[g]:
            inp[g, r] = 0
    t = _dev(inp)
    stt = torch.full((G,), -1, dtype=torch.int8, device="cuda")
    enc.reconstruct_batch(t, torch.as_tensor(words.view(np.int64)).cuda(), shard_size=S, status=stt)
    got = t.cpu().numpy()
    for g in range(G):
        rows = [None if r in erased[g] else bytearray(want[g, r, :S].tobytes()) for r in range(n)]
        err = rs_ref.reconstruct_group(M, d, p, rows)
        assert int(stt[g]) == (0 if err is None else fec.ErrTooFewShards.code)
        for r in range(n):
            exp = bytes(rows[r]) if err is None else inp[g, r, :S].tobytes()
            assert got[g, r, :S].tobytes() == exp, (g, r)


@pytest.mark.parametrize("S", [9000, 8999, 8193, 1, 15, 17, 1350, 4096])
@pytest.mark.parametrize("shard_major", [False, True])
def test_jumbo_encode_four_russians_vs_oracle(gpu, S, shard_major):
    """The (32,8) encode runs the compile-time network in Four-Russians form
    (k_encode_frs): parity bit-exact vs the C oracle for full and partial tail
    chunks, group-major and planar, and padding past S untouched."""
    d, p, G = 32, 8, 70
    n = d + p
    pitch = (S + 15) // 16 * 16
    host = _rand(G, n, pitch, 9000 + S).numpy()
    want = host.copy()
    rs_ref.c_encode(d, p, want, S=S)
    want[:, d:, S:] = host[:, d:, S:]  # the kernel leaves padding as it was
    enc = fec.New(d, p)
    if shard_major:
        t = _dev(np.ascontiguousarray(host.transpose(1, 0, 2)))
        enc.encode_batch(t, shard_size=S, shard_major=True)
        got = t.cpu().numpy().transpose(1, 0, 2)
    else:
        t = _dev(host)
        enc.encode_batch(t, shard_size=S)
        got = t.cpu().numpy()
    assert np.array_equal(got, want)


@pytest.mark.parametrize("d,p,S,where,data_only", [
    (10, 3, 1476, "pinned", True),    # the FEC object's batched recovery: pooled 1476-B buffers
    (10, 3, 1476, "pinned", False),
    (10, 3, 1470, "device", False),
    (20, 4, 1000, "device", False),   # d+p > 16: per-group descriptors (k_prepare)
    (5, 3, 17, "pinned", True),       # a 1-byte tail chunk
    (40, 8, 300, "device", False),    # d > 8 inputs and e up to 8 outputs in one pass each
])
def test_reconstruct_rows_vs_oracle(gpu, d, p, S, where, data_only):
    """ugo_fec_reconstruct_rows: every row of every group at its own address in
    a shuffled pool of slots (device memory, or pinned host memory read in
    place over PCIe), absent rows NULL, erased rows' old slots holding garbage.
    Recovered rows, statuses and untouched slots vs the oracle."""
    n, G = d + p, 300
    rng = np.random.default_rng(d * 1000 + S)
    data = rng.integers(0, 256, (G, n, S), dtype=np.uint8)
    rs_ref.c_encode(d, p, data)
    ne = rng.integers(0, p + 2, G)  # p+1 erasures: too few shards
    masks = np.full(G, (1 << n) - 1, np.uint64)
    for g in range(G):
        for r in rng.choice(n, int(ne[g]), replace=False):
            masks[g] &= ~np.uint64(1 << int(r))
    sp = (S + 15) // 16 * 16 + 16 * int(rng.integers(0, 3))
    nslots = G * n + 37
    slot_of = rng.permutation(nslots)[:G * n].reshape(G, n)
    enc = fec.New(d, p)
    pool_host = rng.integers(0, 256, (nslots, sp), dtype=np.uint8)
    for g in range(G):
        for r in range(n):
            if (int(masks[g]) >> r) & 1:
                pool_host[slot_of[g, r], :S] = data[g, r]
    keep = []
    if where == "pinned":
        raw = fec.host_alloc(nslots * sp)
        keep.append(raw)
        pool = raw.reshape(nslots, sp)
        pool[:] = pool_host
        base = enc.device_address(pool.ctypes.data)
        rows_raw = fec.host_alloc(G * n * 8)
        keep.append(rows_raw)
        rows = rows_raw.view(np.int64).reshape(G, n)
        pres_raw = fec.host_alloc(G * 8)
        keep.append(pres_raw)
        present = pres_raw.view(np.uint64)
        present[:] = masks
    else:
        pool = torch.from_numpy(pool_host).cuda()
        base = pool.data_ptr()
        rows = np.zeros((G, n), np.int64)
        present = _masks_to_dev(masks)
    try:
        for g in range(G):
            for r in range(n):
                rows[g, r] = base + int(slot_of[g, r]) * sp if (int(masks[g]) >> r) & 1 else 0
        bad_g = int(np.nonzero((ne > 0) & (ne <= p))[0][0])  # a recoverable group with a misaligned survivor
        first_present = next(r for r in range(n) if (int(masks[bad_g]) >> r) & 1)
        rows[bad_g, first_present] += 1
        rows_arg = rows if where == "pinned" else torch.from_numpy(rows).cuda()
        out = torch.full((p, G, sp), 0xA5, dtype=torch.uint8, device="cuda")
        st = torch.full((G,), -1, dtype=torch.int8, device="cuda")
        enc.reconstruct_rows(rows_arg, present, out, S, data_only=data_only, status=st)
        torch.cuda.synchronize()
        o = out.cpu().numpy()
        stv = st.cpu().numpy()
        want_rc = data.copy()
        erased = _erase(want_rc, masks, n)
        rc, want_st = rs_ref.c_reconstruct(d, p, erased, masks, data_only=data_only)
        for g in range(G):
            er = [r for r in range(n) if not (int(masks[g]) >> r) & 1]
            if g == bad_g:
                assert stv[g] == 6 and (o[:, g] == 0xA5).all(), g
                continue
            assert stv[g] == want_st[g], (g, stv[g], want_st[g])
            if want_st[g] != 0:
                assert (o[:, g] == 0xA5).all(), g
                continue
            outs = [r for r in er if r < d] if data_only else er
            for i, r in enumerate(outs):
                assert np.array_equal(o[i, g, :S], data[g, r]), (g, i, r)
                assert (o[i, g, S:] == 0xA5).all(), (g, i)  # padding of the output slot untouched
            assert (o[len(outs):, g] == 0xA5).all(), g
        # the pool is only read
        now = pool if where == "pinned" else pool.cpu().numpy()
        assert np.array_equal(np.asarray(now), pool_host)
    finally:
        del pool
        for k in keep:
            fec.host_free(k)
