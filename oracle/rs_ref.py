"""ORACLE -- TEST INFRASTRUCTURE ONLY (pure-Python mirror of oracle/rs_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker.  The product path never does.

An *independent* second restatement of the klauspost/reedsolomon arithmetic
that ugo/fec.go delegates to (import ugo/fec.go:9, New at :59, Reconstruct at
:202, Encode at :238).  It deliberately uses a different multiply (bitwise
shift-and-reduce by the field polynomial 0x11D) from the C oracle (log/exp
tables), so agreement between the two cross-checks both.  Pure-Python loops:
use it for small cases only.

The loader for the compiled C oracle also lives here (`load_c_oracle`).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

POLY = 0x11D

_HERE = os.path.dirname(os.path.abspath(__file__))


def gf_mul(a: int, b: int) -> int:
    """Russian-peasant multiply in GF(2^8) mod x^8+x^4+x^3+x^2+1 [upstream galois.go]."""
    r = 0
    a &= 0xFF
    b &= 0xFF
    while b:
        if b & 1:
            r ^= a
        b >>= 1
        a <<= 1
        if a & 0x100:
            a ^= POLY
    return r


def gf_pow(a: int, n: int) -> int:
    """galExp(a, n): 1 when n == 0 (also for a == 0), 0 when a == 0 and n > 0."""
    if n == 0:
        return 1
    if a == 0:
        return 0
    r = 1
    for _ in range(n):
        r = gf_mul(r, a)
    return r


def gf_inv(a: int) -> int:
    if a == 0:
        raise ZeroDivisionError
    # a^254 = a^-1 in GF(2^8)
    return gf_pow(a, 254)


class Singular(Exception):
    pass


def mat_mul(A, B):
    r, k, c = len(A), len(B), len(B[0])
    out = [[0] * c for _ in range(r)]
    for i in range(r):
        for j in range(c):
            v = 0
            for t in range(k):
                v ^= gf_mul(A[i][t], B[t][j])
            out[i][j] = v
    return out


def mat_inv(A):
    """Gauss-Jordan over GF(2^8) [upstream matrix.go Invert]."""
    n = len(A)
    a = [list(row) + [1 if i == j else 0 for j in range(n)] for i, row in enumerate(A)]
    for r in range(n):
        if a[r][r] == 0:
            for below in range(r + 1, n):
                if a[below][r]:
                    a[r], a[below] = a[below], a[r]
                    break
            else:
                raise Singular()
        s = gf_inv(a[r][r])
        a[r] = [gf_mul(s, v) for v in a[r]]
        for o in range(n):
            if o != r and a[o][r]:
                f = a[o][r]
                a[o] = [x ^ gf_mul(f, y) for x, y in zip(a[o], a[r])]
    return [row[n:] for row in a]


def build_matrix(d: int, p: int):
    """buildMatrix(d, d+p) [upstream]: Vandermonde times inverse of its top."""
    n = d + p
    V = [[gf_pow(r, c) for c in range(d)] for r in range(n)]
    return mat_mul(V, mat_inv(V[:d]))


def encode_group(M, d: int, p: int, rows):
    """rows: list of n bytearrays of equal length; writes parity rows in place."""
    S = len(rows[0])
    for i in range(p):
        out = bytearray(S)
        for k in range(d):
            c = M[d + i][k]
            src = rows[k]
            for j in range(S):
                out[j] ^= gf_mul(c, src[j])
        rows[d + i][:] = out


def reconstruct_group(M, d: int, p: int, rows, data_only=False):
    """rows: list of n entries, None/empty = erased.  Mirrors upstream
    Reconstruct: first d present in index order, two-stage rebuild.
    Returns 'ErrTooFewShards' or None; fills erased entries in place."""
    n = d + p
    present = [r is not None and len(r) != 0 for r in rows]
    npres = sum(present)
    if npres == n or (data_only and all(present[:d])):
        return None
    if npres < d:
        return "ErrTooFewShards"
    S = len(next(r for r in rows if r is not None and len(r) != 0))
    valid = [i for i in range(n) if present[i]][:d]
    inv = mat_inv([M[v] for v in valid])
    for r in range(d):
        if not present[r]:
            out = bytearray(S)
            for k, v in enumerate(valid):
                c = inv[r][k]
                for j in range(S):
                    out[j] ^= gf_mul(c, rows[v][j])
            rows[r] = out
    if not data_only:
        for r in range(d, n):
            if not present[r]:
                out = bytearray(S)
                for k in range(d):
                    c = M[r][k]
                    for j in range(S):
                        out[j] ^= gf_mul(c, rows[k][j])
                rows[r] = out
    return None


# ---------------------------------------------------------------- C oracle
_lib = None


def build_c_oracle() -> str:
    """Compile oracle/rs_oracle.c -> oracle/librs_oracle.so (gcc, -O2)."""
    so = os.path.join(_HERE, "librs_oracle.so")
    src = os.path.join(_HERE, "rs_oracle.c")
    if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE, "librs_oracle.so"])
    return so


def load_c_oracle():
    global _lib
    if _lib is not None:
        return _lib
    so = build_c_oracle()
    lib = ctypes.CDLL(so)
    u8p = ctypes.POINTER(ctypes.c_uint8)
    sz = ctypes.c_size_t
    lib.oracle_init.restype = None
    lib.oracle_gf_mul.restype = ctypes.c_uint8
    lib.oracle_gf_mul.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
    lib.oracle_gf_exp.restype = ctypes.c_uint8
    lib.oracle_gf_exp.argtypes = [ctypes.c_uint8, ctypes.c_int]
    lib.oracle_invert.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    lib.oracle_matmul.argtypes = [ctypes.c_int] * 3 + [ctypes.c_void_p] * 3
    lib.oracle_matmul.restype = None
    lib.oracle_matrix.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    lib.oracle_encode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, sz, sz, sz]
    lib.oracle_encode_mt.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, sz, sz, sz, ctypes.c_int]
    lib.oracle_reconstruct.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                       sz, sz, sz, ctypes.c_int, ctypes.c_void_p]
    lib.oracle_reconstruct_mt.argtypes = lib.oracle_reconstruct.argtypes + [ctypes.c_int]
    lib.oracle_check_shards.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(sz)]
    lib.oracle_check_geometry.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.oracle_fill.argtypes = [ctypes.c_void_p, ctypes.c_int, sz, sz, sz, ctypes.c_uint64, ctypes.c_int]
    lib.oracle_fill.restype = None
    lib.oracle_set_simd.argtypes = [ctypes.c_int]
    lib.oracle_simd_level.argtypes = []
    lib.oracle_init()
    del u8p
    _lib = lib
    return lib


def set_simd(level: int) -> int:
    """CPU-baseline SIMD level of the C oracle (0 scalar, 1 AVX2, 2 AVX-512
    GFNI, -1 best available); returns the level in effect."""
    return load_c_oracle().oracle_set_simd(level)


SIMD_NAMES = {0: "scalar", 1: "avx2-nibble-pshufb", 2: "avx512-gfni-affine"}


def _ptr(a: np.ndarray):
    assert a.flags["C_CONTIGUOUS"]
    return ctypes.c_void_p(a.ctypes.data)


def c_matrix(d: int, p: int) -> np.ndarray:
    lib = load_c_oracle()
    out = np.zeros(((d + p), d), dtype=np.uint8)
    rc = lib.oracle_matrix(d, p, _ptr(out))
    if rc:
        raise ValueError(f"oracle_matrix rc={rc}")
    return out


def c_invert(m: np.ndarray) -> np.ndarray:
    lib = load_c_oracle()
    m = np.ascontiguousarray(m, dtype=np.uint8)
    out = np.zeros_like(m)
    rc = lib.oracle_invert(m.shape[0], _ptr(m), _ptr(out))
    if rc:
        raise Singular()
    return out


def c_encode(d: int, p: int, shards: np.ndarray, S: int | None = None, threads: int = 1) -> int:
    """shards: uint8 [G, d+p, pitch], modified in place."""
    lib = load_c_oracle()
    G, n, pitch = shards.shape
    assert n == d + p
    return lib.oracle_encode_mt(d, p, _ptr(shards), G, pitch if S is None else S, pitch, threads)


def c_reconstruct(d: int, p: int, shards: np.ndarray, present: np.ndarray, S: int | None = None,
                  data_only: bool = False, threads: int = 1):
    """Returns (rc, status[G])."""
    lib = load_c_oracle()
    G, n, pitch = shards.shape
    present = np.ascontiguousarray(present, dtype=np.uint64)
    status = np.zeros(G, dtype=np.int8)
    rc = lib.oracle_reconstruct_mt(d, p, _ptr(shards), _ptr(present), G, pitch if S is None else S,
                                   pitch, int(data_only), _ptr(status), threads)
    return rc, status


def c_fill(shards: np.ndarray, S: int, seed: int, rows: int | None = None):
    lib = load_c_oracle()
    G, n, pitch = shards.shape
    lib.oracle_fill(_ptr(shards), n, G, S, pitch, ctypes.c_uint64(seed), n if rows is None else rows)
