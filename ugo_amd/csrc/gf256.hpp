// gf256.hpp -- GF(2^8) field and the Reed-Solomon code matrix used by
// jflyup/ugo's FEC (ugo/fec.go:59 -> klauspost/reedsolomon.New(d, p)).
//
// Field: x^8 + x^4 + x^3 + x^2 + 1 (0x11D), generator 2.  Code: systematic
// matrix M = V * inverse(V[0:d]) with V[r][c] = r^c (0^0 = 1), (d+p) x d.
// Everything here is constexpr so the hot geometries get their coefficients
// folded into the kernels at compile time (fec_kernels.hip), and the same code
// builds runtime matrices / decode descriptors on the host (ugo_fec.cpp).
#pragma once
#include <cstddef>
#include <cstdint>

namespace ugo {
namespace gf {

struct Tables {
  uint8_t exp[512];
  uint8_t log[256];
};

constexpr Tables make_tables() {
  Tables t{};
  int x = 1;
  for (int i = 0; i < 255; ++i) {
    t.exp[i] = static_cast<uint8_t>(x);
    t.log[x] = static_cast<uint8_t>(i);
    x <<= 1;
    if (x & 0x100) x ^= 0x11d;
  }
  for (int i = 255; i < 512; ++i) t.exp[i] = t.exp[i - 255];
  t.log[0] = 0;
  return t;
}

inline constexpr Tables kTables = make_tables();

constexpr uint8_t mul(uint8_t a, uint8_t b) {
  if (a == 0 || b == 0) return 0;
  return kTables.exp[kTables.log[a] + kTables.log[b]];
}

constexpr uint8_t inv(uint8_t a) {  // a != 0
  return kTables.exp[(255 - kTables.log[a]) % 255];
}

constexpr uint8_t pow(uint8_t a, int n) {
  if (n == 0) return 1;
  if (a == 0) return 0;
  return kTables.exp[(kTables.log[a] * n) % 255];
}

// In-place Gauss-Jordan inverse of an n x n row-major matrix `a` into `out`.
// `work` must hold 2*n*n bytes.  Returns false if singular.
constexpr bool invert(int n, const uint8_t* a, uint8_t* out, uint8_t* work) {
  const int w = 2 * n;
  for (int r = 0; r < n; ++r)
    for (int c = 0; c < w; ++c)
      work[r * w + c] = c < n ? a[r * n + c] : static_cast<uint8_t>(c - n == r ? 1 : 0);
  for (int r = 0; r < n; ++r) {
    if (work[r * w + r] == 0) {
      int b = r + 1;
      while (b < n && work[b * w + r] == 0) ++b;
      if (b == n) return false;
      for (int c = 0; c < w; ++c) {
        uint8_t t = work[r * w + c];
        work[r * w + c] = work[b * w + c];
        work[b * w + c] = t;
      }
    }
    const uint8_t s = inv(work[r * w + r]);
    for (int c = 0; c < w; ++c) work[r * w + c] = mul(s, work[r * w + c]);
    for (int o = 0; o < n; ++o) {
      if (o == r) continue;
      const uint8_t f = work[o * w + r];
      if (f)
        for (int c = 0; c < w; ++c) work[o * w + c] ^= mul(f, work[r * w + c]);
    }
  }
  for (int r = 0; r < n; ++r)
    for (int c = 0; c < n; ++c) out[r * n + c] = work[r * w + n + c];
  return true;
}

// (d+p) x d systematic encoding matrix into `m`; `scratch` >= (d+p)*d + 3*d*d.
constexpr bool build_matrix(int d, int p, uint8_t* m, uint8_t* scratch) {
  const int n = d + p;
  uint8_t* V = scratch;              // n x d
  uint8_t* Ti = V + n * d;           // d x d
  uint8_t* work = Ti + d * d;        // 2 d x d
  for (int r = 0; r < n; ++r)
    for (int c = 0; c < d; ++c) V[r * d + c] = pow(static_cast<uint8_t>(r), c);
  if (!invert(d, V, Ti, work)) return false;
  for (int r = 0; r < n; ++r)
    for (int c = 0; c < d; ++c) {
      uint8_t v = 0;
      for (int k = 0; k < d; ++k) v ^= mul(V[r * d + k], Ti[k * d + c]);
      m[r * d + c] = v;
    }
  return true;
}

// Compile-time matrix for the geometries the kernels specialise on.
// Split multiplication tables for the v_perm_b32 kernels: for coefficient c,
// 8 dwords at out + 32*c: T0[j] = c*j (j < 8), T1[j] = c*(j << 3) (j < 8),
// T2[j] = c*(j << 6) (j < 4), packed little-endian (T0 lo/hi, T1 lo/hi, T2,
// 3 zero dwords), so c*x = T0[x & 7] ^ T1[(x >> 3) & 7] ^ T2[x >> 6].
inline void perm_tables(uint8_t* out) {
  for (int c = 0; c < 256; ++c) {
    uint8_t* t = out + 32 * c;
    for (int j = 0; j < 32; ++j) t[j] = 0;
    for (int j = 0; j < 8; ++j) {
      t[j] = mul(static_cast<uint8_t>(c), static_cast<uint8_t>(j));
      t[8 + j] = mul(static_cast<uint8_t>(c), static_cast<uint8_t>(j << 3));
    }
    for (int j = 0; j < 4; ++j) t[16 + j] = mul(static_cast<uint8_t>(c), static_cast<uint8_t>(j << 6));
  }
}

template <int D, int P>
struct CodeMatrix {
  static constexpr int N = D + P;
  uint8_t m[N * D];
  constexpr CodeMatrix() : m{} {
    uint8_t scratch[N * D + 3 * D * D] = {};
    build_matrix(D, P, m, scratch);
  }
  constexpr uint8_t at(int r, int c) const { return m[r * D + c]; }
};

template <int D, int P>
struct Code {
  static constexpr CodeMatrix<D, P> M{};
};

}  // namespace gf
}  // namespace ugo
