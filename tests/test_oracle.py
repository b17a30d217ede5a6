"""CPU: pin the oracle (test infrastructure) before trusting it.

1. Recalled upstream klauspost known-answer vectors (tests/golden/klauspost_kat.json)
   for both restatements (C: log/exp tables; Python: shift-and-reduce).
2. Committed golden fixtures match their manifest and are reproduced by the C oracle.
3. Algebraic properties of the code ugo/fec.go:59 builds: systematic, MDS
   (every d-row sub-matrix invertible), round trips, linearity, column independence.
"""
import hashlib
import itertools
import json
import os

import numpy as np
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st
import pytest

import rs_ref

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def kat():
    return json.load(open(os.path.join(GOLD, "klauspost_kat.json")))


@pytest.fixture(scope="module")
def fx():
    return dict(np.load(os.path.join(GOLD, "fixtures_v1.npz")))


def test_kat_galois(kat):
    lib = rs_ref.load_c_oracle()
    for a, b, want in kat["gal_multiply"]:
        assert rs_ref.gf_mul(a, b) == want
        assert lib.oracle_gf_mul(a, b) == want
    for a, n, want in kat["gal_exp"]:
        assert rs_ref.gf_pow(a, n) == want
        assert lib.oracle_gf_exp(a, n) == want
    inp = kat["gal_mul_slice_input"]
    for c, want in kat["gal_mul_slice"].items():
        got = [rs_ref.gf_mul(int(c), x) for x in inp[: len(want)]]
        assert got == want
        assert [lib.oracle_gf_mul(int(c), x) for x in inp[: len(want)]] == want


def _clmul_mod_11d(a, b):
    """GF(2^8) product by carry-less multiply, then reduction by 0x11D: a
    third computation, independent of both restatements' tables."""
    r = 0
    for i in range(8):
        if (b >> i) & 1:
            r ^= a << i
    for bit in range(15, 7, -1):
        if (r >> bit) & 1:
            r ^= 0x11D << (bit - 8)
    return r


def test_kat_galois_recalled_tail_refuted(kat):
    """The recalled galMulSlice(177) tail disagrees with both restatements.
    Multiplication by 177 is fully determined once the field (polynomial
    0x11D, pinned by every other vector) is fixed, so a third, table-free
    computation settles it: the restatements are right and the recalled
    values are a memory error, kept in the fixture only as a record."""
    disp = kat["gal_mul_slice_disputed"]
    c, inp = disp["coefficient"], disp["inputs"]
    lib = rs_ref.load_c_oracle()
    field = [_clmul_mod_11d(c, x) for x in inp]
    assert [rs_ref.gf_mul(c, x) for x in inp] == [lib.oracle_gf_mul(c, x) for x in inp] == field
    assert field == disp["restatements"]
    assert field != disp["recalled"]
    # the same table-free product agrees with every pinned multiply vector
    for a, b, want in kat["gal_multiply"]:
        assert _clmul_mod_11d(a, b) == want


def test_kat_matrix(kat):
    mm = kat["matrix_multiply"]
    assert rs_ref.mat_mul(mm["a"], mm["b"]) == mm["out"]
    for case in kat["matrix_inverse"]:
        assert rs_ref.mat_inv(case["in"]) == case["out"]
        assert rs_ref.c_invert(np.array(case["in"], np.uint8)).tolist() == case["out"]
    for m in kat["matrix_singular"]:
        with pytest.raises(rs_ref.Singular):
            rs_ref.mat_inv(m)
        with pytest.raises(rs_ref.Singular):
            rs_ref.c_invert(np.array(m, np.uint8))


def test_kat_one_encode(kat):
    c = kat["one_encode"]
    d, p = c["d"], c["p"]
    sh = np.zeros((1, d + p, 2), np.uint8)
    sh[0, :d] = c["data"]
    assert rs_ref.c_encode(d, p, sh) == 0
    assert sh[0, d:].tolist() == c["parity"]
    rows = [bytearray(bytes(r)) for r in c["data"]] + [bytearray(2) for _ in range(p)]
    rs_ref.encode_group(rs_ref.build_matrix(d, p), d, p, rows)
    assert [list(r) for r in rows[d:]] == c["parity"]


def test_fixture_manifest(fx):
    man = json.load(open(os.path.join(GOLD, "fixtures_v1.manifest.json")))
    assert set(man) == set(fx)
    for k, v in fx.items():
        assert hashlib.sha256(np.ascontiguousarray(v).tobytes()).hexdigest() == man[k]["sha256"], k


def test_fixtures_reproduced_by_oracle(fx):
    for key, m in fx.items():
        if key.startswith("matrix_"):
            _, d, p = key.split("_")
            assert np.array_equal(rs_ref.c_matrix(int(d), int(p)), m)
    enc = np.concatenate([fx["g10_enc_data"], np.zeros_like(fx["g10_enc_parity"])], axis=1)
    rs_ref.c_encode(10, 3, enc)
    assert np.array_equal(enc[:, 10:], fx["g10_enc_parity"])
    out = fx["g10_in"].copy()
    rc, st = rs_ref.c_reconstruct(10, 3, out, fx["g10_mask"])
    assert rc == 0 and np.array_equal(out, fx["g10_out"])
    out = fx["g10x_in"].copy()
    rs_ref.c_reconstruct(10, 3, out, fx["g10x_mask"])
    assert np.array_equal(out, fx["g10x_out"])
    j = fx["g32_out"].copy()
    mk = int(fx["g32_mask"][0])
    for r in range(40):
        if not (mk >> r) & 1:
            j[0, r] = 0
    rs_ref.c_reconstruct(32, 8, j, fx["g32_mask"])
    assert np.array_equal(j, fx["g32_out"])


def test_matrix_10_3_survey_rows():
    # SURVEY.md §8a lists the (10,3) parity rows
    m = rs_ref.c_matrix(10, 3)
    assert m[10].tolist() == [129, 150, 175, 184, 210, 196, 254, 232, 3, 2]
    assert m[11].tolist() == [150, 129, 184, 175, 196, 210, 232, 254, 2, 3]
    assert m[12].tolist() == [191, 214, 98, 10, 6, 111, 223, 183, 5, 4]


@pytest.mark.parametrize("d,p", [(10, 3), (5, 5), (4, 2), (12, 4)])
def test_systematic_and_mds(d, p):
    m = rs_ref.c_matrix(d, p)
    assert np.array_equal(m[:d], np.eye(d, dtype=np.uint8))
    for rows in itertools.combinations(range(d + p), d):  # C(13,10) = 286 for (10,3)
        rs_ref.c_invert(m[list(rows)])  # raises Singular if not MDS


def test_mds_sampled_32_8():
    m = rs_ref.c_matrix(32, 8)
    rng = np.random.default_rng(1)
    for _ in range(200):
        rows = np.sort(rng.choice(40, 32, replace=False))
        rs_ref.c_invert(m[rows])


def test_round_trip_every_pattern_10_3():
    d, p, n, S = 10, 3, 13, 40
    rng = np.random.default_rng(7)
    masks = [m for m in range(1 << n)]
    G = len(masks)
    sh = np.zeros((G, n, S), np.uint8)
    sh[:, :d] = rng.integers(0, 256, size=(G, d, S), dtype=np.uint8)
    rs_ref.c_encode(d, p, sh)
    want = sh.copy()
    for g, m in enumerate(masks):
        for r in range(n):
            if not (m >> r) & 1:
                sh[g, r] = 0
    rc, st = rs_ref.c_reconstruct(d, p, sh, np.array(masks, np.uint64))
    for g, m in enumerate(masks):
        if bin(m).count("1") >= d:
            assert st[g] == 0
            assert np.array_equal(sh[g], want[g]), m
        else:
            assert st[g] == 3  # ErrTooFewShards


def test_linearity_and_columns():
    d, p, S = 10, 3, 64
    rng = np.random.default_rng(3)
    a = np.zeros((1, 13, S), np.uint8)
    b = np.zeros((1, 13, S), np.uint8)
    a[0, :d] = rng.integers(0, 256, (d, S), dtype=np.uint8)
    b[0, :d] = rng.integers(0, 256, (d, S), dtype=np.uint8)
    ab = a ^ b
    for x in (a, b, ab):
        rs_ref.c_encode(d, p, x)
    assert np.array_equal(ab, a ^ b)
    # column independence: encoding a column window equals the window of the encoding
    w = np.ascontiguousarray(a[:, :, 17:41])
    w2 = w.copy()
    w2[:, d:] = 0
    rs_ref.c_encode(d, p, w2)
    assert np.array_equal(w2, w)


def test_python_mirror_agrees_with_c():
    rng = np.random.default_rng(11)
    for d, p in [(3, 2), (10, 3)]:
        M = rs_ref.build_matrix(d, p)
        assert np.array_equal(np.array(M, np.uint8), rs_ref.c_matrix(d, p))
        rows = [bytearray(rng.integers(0, 256, 24, dtype=np.uint8).tobytes()) for _ in range(d)] + \
               [bytearray(24) for _ in range(p)]
        rs_ref.encode_group(M, d, p, rows)
        arr = np.array([list(r) for r in rows], np.uint8)[None]
        c = arr.copy()
        c[:, d:] = 0
        rs_ref.c_encode(d, p, c)
        assert np.array_equal(c, arr)


@settings(max_examples=120, deadline=None, derandomize=True, suppress_health_check=[HealthCheck.too_slow])
@given(d=st.integers(1, 16), p=st.integers(1, 8), S=st.integers(1, 40), seed=st.integers(0, 2**32 - 1),
       data=st.data())
def test_restatements_agree_on_random_codes(d, p, S, seed, data):
    """The two independent restatements (C, table multiply; Python,
    shift-and-reduce) agree on random geometries, data and erasure patterns --
    encode, then Reconstruct of any pattern with >= d survivors (first d present
    rows), data-only as well -- and the round trip is the identity."""
    n = d + p
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 256, (1, n, S), dtype=np.uint8)
    rs_ref.c_encode(d, p, a)
    M = rs_ref.build_matrix(d, p)
    rows = [bytearray(a[0, r].tobytes()) for r in range(n)]
    chk = [bytearray(x) for x in rows]
    rs_ref.encode_group(M, d, p, chk)
    assert chk == rows
    e = data.draw(st.integers(0, p), label="erasures")
    erased = sorted(data.draw(st.permutations(list(range(n))), label="order")[:e])
    mask = np.array([((1 << n) - 1) ^ sum(1 << r for r in erased)], np.uint64)
    for data_only in (False, True):
        b = a.copy()
        b[0, erased] = 0
        rc, st_ = rs_ref.c_reconstruct(d, p, b, mask, data_only=data_only)
        py = [None if r in erased else bytearray(rows[r]) for r in range(n)]
        assert rs_ref.reconstruct_group(M, d, p, py, data_only=data_only) is None
        for r in range(n):
            if r in erased and (data_only and r >= d):
                continue  # data-only leaves erased parity rows alone
            assert b[0, r].tobytes() == rows[r] == bytes(py[r]), (d, p, r, data_only)


def test_oracle_errors():
    lib = rs_ref.load_c_oracle()
    assert lib.oracle_check_geometry(0, 3) == 1
    assert lib.oracle_check_geometry(10, -1) == 1
    assert lib.oracle_check_geometry(200, 57) == 2
    import ctypes
    lens = (ctypes.c_size_t * 3)(4, 0, 4)
    out = ctypes.c_size_t()
    assert lib.oracle_check_shards(3, lens, 1, ctypes.byref(out)) == 0 and out.value == 4
    assert lib.oracle_check_shards(3, lens, 0, ctypes.byref(out)) == 5
    lens = (ctypes.c_size_t * 2)(0, 0)
    assert lib.oracle_check_shards(2, lens, 1, ctypes.byref(out)) == 4


@pytest.mark.parametrize("d,p,S", [(10, 3, 1350), (32, 8, 9000), (5, 3, 77), (17, 7, 1)])
def test_simd_baseline_levels_match_scalar(d, p, S):
    """The SIMD forms used only for the timed CPU baseline (AVX2 nibble tables,
    AVX-512 GFNI) reproduce the scalar checker byte for byte."""
    n = d + p
    rng = np.random.default_rng(d * 100 + S)
    base = rng.integers(0, 256, (6, n, S), dtype=np.uint8)
    masks = np.full(6, (1 << n) - 1, np.uint64)
    for g in range(6):
        for r in rng.choice(n, p, replace=False):
            masks[g] &= ~np.uint64(1 << int(r))
    outs = []
    try:
        for level in (0, 1, 2):
            got = rs_ref.set_simd(level)
            sh = base.copy()
            rs_ref.c_encode(d, p, sh)
            enc = sh.copy()
            sh[:, :, :] = np.where(((masks[:, None] >> np.arange(n, dtype=np.uint64)) & 1).astype(bool)[:, :, None], enc, 0)
            rs_ref.c_reconstruct(d, p, sh, masks)
            outs.append((got, enc, sh))
    finally:
        rs_ref.set_simd(0)
    for got, enc, sh in outs[1:]:
        assert np.array_equal(enc, outs[0][1]), f"level {got} encode"
        assert np.array_equal(sh, outs[0][2]), f"level {got} reconstruct"
        assert np.array_equal(sh, outs[0][1])
