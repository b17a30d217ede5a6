"""Generate the committed golden fixtures (tests/golden/fixtures_v1.npz).

Run from the repo root:  python tests/golden/make_golden.py

Every expected output here is produced by the C restatement (oracle/rs_oracle.c)
and independently re-derived by the pure-Python mirror (oracle/rs_ref.py) before
it is written; the script aborts on any disagreement.  Both restatements are
first pinned against the recalled upstream klauspost known-answer vectors in
tests/golden/klauspost_kat.json (see test_oracle.py).  The reference repo holds
no FEC test of its own, so these fixtures are "parity unpinned" with respect to
the reference Go code -- they pin the build to the upstream
algorithm that ugo/fec.go:59/202/238 delegates to.

Contents (all uint8 unless noted):
  matrix_D_P            (D+P) x D encoding matrices for the geometries used
  g10_in / g10_out      4 groups of (10+3)x1350: g10_in has erased rows zeroed,
                        g10_out is the expected Reconstruct result; g10_mask (u64)
  g10_enc_data/_parity  Encode case: data rows -> expected parity rows
  g10x_in / g10x_out    "inconsistent" groups (rows are NOT a codeword, like
                        ugo's stale pool tails, ugo/fec.go:84-87): Reconstruct
                        must still match bit-for-bit because survivor selection
                        (first d present, index order) is fixed
  g32_out / g32_mask    1 jumbo group (32+8)x9000 with 8 mixed erasures
                        (input = g32_out with the erased rows zeroed)
  calcecc_*             ugo calcECC window: 13 x 1476-B buffers, offset 6,
                        maxlen 1100 -> parity written only in [6, 1100)
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import rs_ref  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "fixtures_v1.npz")


def py_check_encode(d, p, grp):
    M = rs_ref.build_matrix(d, p)
    rows = [bytearray(r.tobytes()) for r in grp]
    rs_ref.encode_group(M, d, p, rows)
    return np.array([list(r) for r in rows], dtype=np.uint8)


def py_check_recon(d, p, grp, mask, data_only=False):
    M = rs_ref.build_matrix(d, p)
    rows = [bytearray(grp[r].tobytes()) if (mask >> r) & 1 else None for r in range(d + p)]
    err = rs_ref.reconstruct_group(M, d, p, rows, data_only)
    assert err is None, err
    return np.array([list(r) if r is not None else list(grp[i]) for i, r in enumerate(rows)], dtype=np.uint8)


def main():
    rng = np.random.default_rng(0x5EED)
    fx = {}
    for d, p in [(10, 3), (32, 8), (5, 5), (4, 2), (1, 1), (12, 4)]:
        m = rs_ref.c_matrix(d, p)
        assert np.array_equal(m, np.array(rs_ref.build_matrix(d, p), dtype=np.uint8)), (d, p)
        fx[f"matrix_{d}_{p}"] = m

    # --- (10+3)x1350 encode + reconstruct, 4 groups
    d, p, S = 10, 3, 1350
    n = d + p
    g = np.zeros((4, n, S), np.uint8)
    rs_ref.c_fill(g, S, 0x5EED, rows=d)
    enc = g.copy()
    rs_ref.c_encode(d, p, enc)
    # python cross-check on a column slice (pure python is slow): first 64 cols
    assert np.array_equal(py_check_encode(d, p, enc[0, :, :64].copy()), enc[0, :, :64])
    fx["g10_enc_data"] = enc[:, :d].copy()
    fx["g10_enc_parity"] = enc[:, d:].copy()
    masks = np.array([
        (1 << n) - 1 & ~(1 << 3),                 # one data loss
        (1 << n) - 1 & ~((1 << 0) | (1 << 11)),   # data + parity
        (1 << n) - 1 & ~((1 << 2) | (1 << 5) | (1 << 9)),  # 3 data losses
        (1 << n) - 1 & ~((1 << 10) | (1 << 12)),  # parity only
    ], dtype=np.uint64)
    gin = enc.copy()
    for i, mk in enumerate(masks):
        for r in range(n):
            if not (int(mk) >> r) & 1:
                gin[i, r] = 0
    gout = gin.copy()
    rc, st = rs_ref.c_reconstruct(d, p, gout, masks)
    assert rc == 0 and not st.any()
    assert np.array_equal(gout, enc), "round trip"
    for i in range(4):
        assert np.array_equal(py_check_recon(d, p, gin[i, :, :48].copy(), int(masks[i])), gout[i, :, :48])
    fx["g10_in"], fx["g10_out"], fx["g10_mask"] = gin, gout, masks

    # --- inconsistent rows (not a codeword): exact survivor selection matters
    gx = rng.integers(0, 256, size=(3, n, 96), dtype=np.uint8)
    mx = np.array([
        (1 << n) - 1 & ~(1 << 1),                       # 12 present: survivors 0,2..10
        (1 << n) - 1 & ~((1 << 4) | (1 << 10)),         # survivors 0..3,5..9,11
        (1 << n) - 1 & ~((1 << 0) | (1 << 7) | (1 << 12)),
    ], dtype=np.uint64)
    for i, mk in enumerate(mx):
        for r in range(n):
            if not (int(mk) >> r) & 1:
                gx[i, r] = 0
    gxo = gx.copy()
    rc, st = rs_ref.c_reconstruct(d, p, gxo, mx)
    assert rc == 0
    for i in range(3):
        assert np.array_equal(py_check_recon(d, p, gx[i].copy(), int(mx[i])), gxo[i])
    fx["g10x_in"], fx["g10x_out"], fx["g10x_mask"] = gx, gxo, mx

    # --- jumbo (32+8)x9000, one group, 8 mixed erasures
    d2, p2, S2 = 32, 8, 9000
    n2 = d2 + p2
    j = np.zeros((1, n2, S2), np.uint8)
    rs_ref.c_fill(j, S2, 0x5EED + 1, rows=d2)
    rs_ref.c_encode(d2, p2, j)
    assert np.array_equal(py_check_encode(d2, p2, j[0, :, :16].copy()), j[0, :, :16])
    erased = [1, 5, 9, 17, 31, 33, 36, 39]
    mk = (1 << n2) - 1
    for r in erased:
        mk &= ~(1 << r)
    jin = j.copy()
    jin[0, erased] = 0
    jout = jin.copy()
    rc, st = rs_ref.c_reconstruct(d2, p2, jout, np.array([mk], np.uint64))
    assert rc == 0 and np.array_equal(jout, j)
    fx["g32_out"], fx["g32_mask"] = jout, np.array([mk], np.uint64)  # input = g32_out with erased rows zeroed

    # --- ugo calcECC window (ugo/fec.go:228-243): 13 x 1476 buffers, offset 6,
    # maxlen 1100; bytes outside [6, maxlen) of parity buffers are untouched.
    buf = rng.integers(0, 256, size=(1, 13, 1476), dtype=np.uint8)
    exp = buf.copy()
    win = np.ascontiguousarray(exp[:, :, 6:1100])
    rs_ref.c_encode(10, 3, win)
    exp[:, :, 6:1100] = win
    fx["calcecc_in"], fx["calcecc_out"] = buf, exp

    np.savez_compressed(OUT, **fx)
    man = {k: {"shape": list(v.shape), "dtype": str(v.dtype),
               "sha256": hashlib.sha256(np.ascontiguousarray(v).tobytes()).hexdigest()} for k, v in fx.items()}
    with open(os.path.join(ROOT, "tests", "golden", "fixtures_v1.manifest.json"), "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
