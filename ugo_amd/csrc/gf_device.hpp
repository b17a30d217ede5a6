// gf_device.hpp -- gfx950 device building blocks shared by the FEC kernels
// (fec_kernels.hip) and the TX assembly kernel (tx_kernels.hip): packed
// GF(2^8) xtime, bitop3 XOR forms, 16-byte loads/stores with cache policy,
// and the compile-time coefficient networks (Horner over coefficient bits).
// See fec_kernels.hip's header for the arithmetic.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <utility>

#include "gf256.hpp"

namespace ugo {
namespace kern {

// ---------------------------------------------------------------- helpers
// Block index, optionally XCD-contiguous (SWZ = 1): the hardware deals blocks
// round-robin to the 8 XCDs; remapped, XCD x runs one contiguous range of
// tiles (cdna_hip_programming.md §5.5 T1, nwg % 8 != 0 form).
template <int SWZ>
__device__ __forceinline__ uint32_t block_id() {
  if constexpr (SWZ == 0) {
    return blockIdx.x;
  } else {
    const uint32_t nwg = gridDim.x, b = blockIdx.x;
    const uint32_t q = nwg >> 3, r = nwg & 7u, x = b & 7u;
    return (x < r ? x * (q + 1u) : r * (q + 1u) + (x - r) * q) + (b >> 3);
  }
}

struct V4 {
  uint32_t v[4];
};

__device__ __forceinline__ uint32_t xt1(uint32_t y) {
  const uint32_t s8 = y << 8;
  const uint32_t m = __builtin_amdgcn_perm(s8, y, 0x090b080au);
  return ((y & 0x7f7f7f7fu) << 1) ^ (m & 0x1d1d1d1du);
}

__device__ __forceinline__ void xt4(V4& y) {
#pragma unroll
  for (int j = 0; j < 4; ++j) y.v[j] = xt1(y.v[j]);
}

__device__ __forceinline__ void xor4(V4& y, const V4& x) {
#pragma unroll
  for (int j = 0; j < 4; ++j) y.v[j] ^= x.v[j];
}

// v_bitop3_b32 truth tables (bit index = a*4 + b*2 + c)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // a ^ b ^ c
}
__device__ __forceinline__ uint32_t xor_and(uint32_t y, uint32_t x, uint32_t m) {
  return __builtin_amdgcn_bitop3_b32(y, x, m, 0x78);  // y ^ (x & m)
}

__device__ __forceinline__ void xor4_2(V4& y, const V4& a, const V4& b) {
#pragma unroll
  for (int j = 0; j < 4; ++j) y.v[j] = xor3(y.v[j], a.v[j], b.v[j]);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// NT policy bits: 1 = nontemporal loads, 2 = nontemporal stores (streaming
// data touched once; keeps it from displacing L2 / Infinity-Cache lines)
template <int NT>
__device__ __forceinline__ V4 load16(const uint8_t* p) {
  const u32x4* q = reinterpret_cast<const u32x4*>(p);
  u32x4 v;
  if constexpr (NT & 1) {
    v = __builtin_nontemporal_load(q);
  } else {
    v = *q;
  }
  return V4{{v.x, v.y, v.z, v.w}};
}

// LDS-DMA staging (global_load_lds_dwordx4, MI355X_MICROARCH.md "ldsdma-fill"):
// lane l's 16 bytes at p land at stage + 16*l (the LDS destination is the
// wave-uniform `stage` plus lane*16).  AUX 2 = nontemporal.  The wave must
// wait with lds_dma_wait() before reading the stage.  Measured (tools/
// membench.hip): the planar encode pattern with its 10 row loads through
// LDS-DMA nt moves 6.56 TB/s against 6.26 TB/s with nt register loads.
template <int AUX = 2>
__device__ __forceinline__ void lds_dma16(const uint8_t* p, u32x4* stage) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(p),
                                   (__attribute__((address_space(3))) void*)(stage), 16, 0, AUX);
}

__device__ __forceinline__ void lds_dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ V4 lds16(const u32x4* stage_lane) {
  const u32x4 v = *stage_lane;
  return V4{{v.x, v.y, v.z, v.w}};
}

// The same LDS-DMA as a NON-volatile inline asm with no memory clobber.  The
// builtin, and any volatile asm, counts as a write to memory the compiler
// cannot place, so every uniform load after it loses its no-clobber proof and
// becomes a per-lane vector load instead of a scalar load (k_apply_p's
// coefficient tables: 290 vector loads, 34% slower).  Order comes from data
// instead: each DMA threads `tok` through, and lds_collect consumes it.
// lds_base: the row's stage address in LDS (wave-uniform), for M0.
__device__ __forceinline__ void lds_dma16_nt_asm(const uint8_t* p, uint32_t lds_base, uint32_t& tok) {
  uint32_t keep;
  asm("s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %2, off nt\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep), "+s"(tok)
      : "v"(p), "s"(lds_base));
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return static_cast<uint32_t>(reinterpret_cast<uintptr_t>(p));
}

// Wait for the wave's LDS-DMA (tok: the last lds_dma16_nt_asm's) and read N
// staged rows (1 KiB apart, this lane's 16 B each) in ONE asm unit ending in
// lgkmcnt(0): its outputs are ready when it ends, as the compiler assumes.
template <int N>
__device__ __forceinline__ void lds_collect(V4* x, const u32x4* stage_lane, uint32_t tok) {
  static_assert(N == 8 || N == 10, "lds_collect: 8 or 10 rows");
  const uint32_t ad = lds_addr(stage_lane);
  u32x4 v[10];
  if constexpr (N == 10) {
    asm("s_waitcnt vmcnt(0)\n\t"
        "ds_read_b128 %0, %10\n\t"
        "ds_read_b128 %1, %10 offset:1024\n\t"
        "ds_read_b128 %2, %10 offset:2048\n\t"
        "ds_read_b128 %3, %10 offset:3072\n\t"
        "ds_read_b128 %4, %10 offset:4096\n\t"
        "ds_read_b128 %5, %10 offset:5120\n\t"
        "ds_read_b128 %6, %10 offset:6144\n\t"
        "ds_read_b128 %7, %10 offset:7168\n\t"
        "ds_read_b128 %8, %10 offset:8192\n\t"
        "ds_read_b128 %9, %10 offset:9216\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]),
          "=&v"(v[7]), "=&v"(v[8]), "=&v"(v[9])
        : "v"(ad), "s"(tok));
  } else {
    asm("s_waitcnt vmcnt(0)\n\t"
        "ds_read_b128 %0, %8\n\t"
        "ds_read_b128 %1, %8 offset:1024\n\t"
        "ds_read_b128 %2, %8 offset:2048\n\t"
        "ds_read_b128 %3, %8 offset:3072\n\t"
        "ds_read_b128 %4, %8 offset:4096\n\t"
        "ds_read_b128 %5, %8 offset:5120\n\t"
        "ds_read_b128 %6, %8 offset:6144\n\t"
        "ds_read_b128 %7, %8 offset:7168\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]),
          "=&v"(v[7])
        : "v"(ad), "s"(tok));
  }
#pragma unroll
  for (int k = 0; k < N; ++k) x[k] = V4{{v[k].x, v[k].y, v[k].z, v[k].w}};
}

// store the first nb (1..16) bytes of a chunk
// the first nb (1..15) bytes of a chunk, at any byte address: one store per
// dword, bytes one by one
__device__ __forceinline__ void store_bytes_any(uint8_t* p, const V4& y, uint32_t nb) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t lo = 4u * j;
    if (nb >= lo + 4) {
      *reinterpret_cast<uint32_t*>(p + lo) = y.v[j];
    } else if (nb > lo) {
      const uint32_t w = y.v[j], rem = nb - lo;
      p[lo] = static_cast<uint8_t>(w);
      if (rem >= 2) p[lo + 1] = static_cast<uint8_t>(w >> 8);
      if (rem >= 3) p[lo + 2] = static_cast<uint8_t>(w >> 16);
    }
  }
}

template <int NT>
__device__ __forceinline__ void store16(uint8_t* p, const V4& y, uint32_t nb) {
  if (nb >= 16) {
    const u32x4 v = {y.v[0], y.v[1], y.v[2], y.v[3]};
    if constexpr (NT & 2) {
      __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
    } else {
      *reinterpret_cast<u32x4*>(p) = v;
    }
    return;
  }
  // tail chunk of a row whose length is not a multiple of 16 (rare lanes).
  // One store per dword, bytes one by one: a single 2-dword store + short
  // (the whole dwords' count picked by masks) made the (10,3) encode 1.2%
  // slower (190.9-191.9 vs 188.7-189.1 us, profiles/r3/tail_ab.jsonl).
  store_bytes_any(p, y, nb);
}

// ------------------------------------------------ compile-time coefficients
template <int D, int P, int I, int B, int K>
__device__ __forceinline__ constexpr bool cbit() {
  return ((gf::Code<D, P>::M.at(D + I, K) >> B) & 1) != 0;
}

template <int D, int P, int I, int B, int... K>
__device__ __forceinline__ constexpr bool any_bit(std::integer_sequence<int, K...>) {
  return (cbit<D, P, I, B, K>() || ...);
}

template <int D, int P, int I, int B>
__device__ __forceinline__ constexpr bool any_bit_at_or_above() {
  if constexpr (B > 7) {
    return false;
  } else {
    return any_bit<D, P, I, B>(std::make_integer_sequence<int, D>{}) ||
           any_bit_at_or_above<D, P, I, B + 1>();
  }
}

// The inputs whose coefficient has bit B set, for output I, as a compile-time list.
template <int D, int P, int I, int B>
struct Terms {
  struct List {
    int n;
    int k[D];
  };
  static constexpr List make() {
    List l{};
    for (int k = 0; k < D; ++k)
      if ((gf::Code<D, P>::M.at(D + I, k) >> B) & 1) l.k[l.n++] = k;
    return l;
  }
  static constexpr List L = make();
};

// y ^= x[terms J..], two terms per v_bitop3 (3-input XOR)
template <int D, int P, int I, int B, int J>
__device__ __forceinline__ void cterms(V4& y, const V4* x) {
  constexpr int n = Terms<D, P, I, B>::L.n;
  if constexpr (J + 1 < n) {
    constexpr int k0 = Terms<D, P, I, B>::L.k[J];
    constexpr int k1 = Terms<D, P, I, B>::L.k[J + 1];
    xor4_2(y, x[k0], x[k1]);
    cterms<D, P, I, B, J + 2>(y, x);
  } else if constexpr (J < n) {
    constexpr int k0 = Terms<D, P, I, B>::L.k[J];
    xor4(y, x[k0]);
  }
}

// Horner step for bit B of output I (called for B = 7 .. 0)
template <int D, int P, int I, int B>
__device__ __forceinline__ void chorner(V4& y, const V4* x) {
  constexpr int n = Terms<D, P, I, B>::L.n;
  if constexpr (any_bit_at_or_above<D, P, I, B + 1>()) {
    xt4(y);  // y *= 2
    cterms<D, P, I, B, 0>(y, x);
  } else if constexpr (n > 0) {
    constexpr int k0 = Terms<D, P, I, B>::L.k[0];
    y = x[k0];  // first non-zero bit plane: y was 0
    cterms<D, P, I, B, 1>(y, x);
  }
  if constexpr (B > 0) chorner<D, P, I, B - 1>(y, x);
}

template <int D, int P, int I>
__device__ __forceinline__ V4 cparity(const V4* x) {
  V4 y{{0u, 0u, 0u, 0u}};
  chorner<D, P, I, 7>(y, x);
  return y;
}

// compute and store parity rows one at a time (short live ranges)
template <int D, int P, int NT, int... I>
__device__ __forceinline__ void cparity_store(uint8_t* gp, uint64_t pitch, uint32_t nb, const V4* x,
                                              std::integer_sequence<int, I...>) {
  ((store16<NT>(gp + static_cast<uint64_t>(D + I) * pitch, cparity<D, P, I>(x), nb)), ...);
}

// ---- the same network in Four-Russians form (wide codes, VALU-bound) ----
// Inputs in blocks of 3.  Per dword, the 7 nonzero XOR combinations of each
// block are formed once (4 new values per block: ab, ac, bc, abc), and every
// bit-plane sum T(I, B) then takes ONE combination per block instead of one
// term per input: for (32,8) about 9.5 terms instead of 16 per plane, 64
// planes per dword, against 44 extra XORs per dword for the combinations.
constexpr int kFrBlock = 3;

template <int D, int P, int I, int B, int BK = kFrBlock>
struct FrTerms {
  static constexpr int NB = (D + BK - 1) / BK;
  struct List {
    int n;
    int blk[NB];
    int idx[NB];
  };
  static constexpr List make() {
    List l{};
    for (int bl = 0; bl < NB; ++bl) {
      int v = 0;
      for (int t = 0; t < BK; ++t) {
        const int k = BK * bl + t;
        if (k < D && ((gf::Code<D, P>::M.at(D + I, k) >> B) & 1)) v |= 1 << t;
      }
      if (v) {
        l.blk[l.n] = bl;
        l.idx[l.n] = v;
        ++l.n;
      }
    }
    return l;
  }
  static constexpr List L = make();
};

template <int D, int P, int I, int B, int J, int NB, int BK = kFrBlock>
__device__ __forceinline__ void fr_fold(uint32_t& y, const uint32_t (*c)[1 << BK]) {
  constexpr auto L = FrTerms<D, P, I, B, BK>::L;
  if constexpr (J + 1 < L.n) {
    y = xor3(y, c[L.blk[J]][L.idx[J]], c[L.blk[J + 1]][L.idx[J + 1]]);
    fr_fold<D, P, I, B, J + 2, NB, BK>(y, c);
  } else if constexpr (J < L.n) {
    y ^= c[L.blk[J]][L.idx[J]];
  }
}

template <int D, int P, int I, int B, int NB, int BK = kFrBlock>
__device__ __forceinline__ void fr_horner(uint32_t& y, const uint32_t (*c)[1 << BK]) {
  constexpr auto L = FrTerms<D, P, I, B, BK>::L;
  if constexpr (any_bit_at_or_above<D, P, I, B + 1>()) {
    y = xt1(y);
    fr_fold<D, P, I, B, 0, NB, BK>(y, c);
  } else if constexpr (L.n > 0) {
    y = c[L.blk[0]][L.idx[0]];
    fr_fold<D, P, I, B, 1, NB, BK>(y, c);
  }
  if constexpr (B > 0) fr_horner<D, P, I, B - 1, NB, BK>(y, c);
}

template <int D, int P, int NB, int BK, int... I>
__device__ __forceinline__ void fr_outputs(V4* y, int j, const uint32_t (*c)[1 << BK],
                                           std::integer_sequence<int, I...>) {
  ((y[I].v[j] = 0u, fr_horner<D, P, I, 7, NB, BK>(y[I].v[j], c)), ...);
}

// All P parity chunks of one column chunk, dword by dword (so only one dword's
// combinations are live at a time).
template <int D, int P>
__device__ __forceinline__ void cparity_fr(V4* y, const V4* x) {
  constexpr int NB = (D + kFrBlock - 1) / kFrBlock;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    uint32_t c[NB][8];
#pragma unroll
    for (int bl = 0; bl < NB; ++bl) {
      const int k = kFrBlock * bl;
      const uint32_t a = x[k].v[j];
      const uint32_t b = k + 1 < D ? x[k + 1].v[j] : 0u;
      const uint32_t e = k + 2 < D ? x[k + 2].v[j] : 0u;
      c[bl][0] = 0u;
      c[bl][1] = a;
      c[bl][2] = b;
      c[bl][3] = a ^ b;
      c[bl][4] = e;
      c[bl][5] = a ^ e;
      c[bl][6] = b ^ e;
      c[bl][7] = xor3(a, b, e);
    }
    fr_outputs<D, P, NB, kFrBlock>(y, j, c, std::make_integer_sequence<int, P>{});
  }
}

// Ordering token: `t` (and anything derived from it) is taken to depend on the
// 8 outputs of the previous dword, so the next dword's combinations cannot be
// hoisted above them (the scheduler otherwise builds all four dwords' tables
// at once: ~300 registers).
__device__ __forceinline__ void fr_after(uint32_t& t, const V4* y, int j) {
  asm volatile("" : "+v"(t) : "v"(y[0].v[j]), "v"(y[1].v[j]), "v"(y[2].v[j]), "v"(y[3].v[j]), "v"(y[4].v[j]),
                              "v"(y[5].v[j]), "v"(y[6].v[j]), "v"(y[7].v[j]));
}

// cparity_fr for P = 8 with the dwords forced in sequence: rows [0, GR) are read
// from the wave's LDS stage one dword at a time (addresses behind the token),
// rows [GR, D) come from registers (each register row's dword passes through
// the token too).
template <int D, int P, int GR, int BK = kFrBlock>
__device__ __forceinline__ void cparity_fr_seq(V4* y, V4* x, const uint32_t* stage_lane_dw) {
  static_assert(P == 8, "fr_after takes 8 outputs");
  constexpr int NB = (D + BK - 1) / BK;
  uint32_t tok = 0u;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (j > 0) fr_after(tok, y, j - 1);
    uint32_t xin[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
      if (k < GR) {
        xin[k] = stage_lane_dw[(k * 64) * 4 + j + tok];  // ds_read_b32, lane's dword j of row k
      } else {
        xin[k] = x[k].v[j];
        if (j > 0) asm volatile("" : "+v"(xin[k]) : "v"(tok));
      }
    }
    // c[bl][m] = XOR of the block's inputs t with bit t of m set: each entry
    // is an earlier entry (lowest bit of m cleared) plus one input
    uint32_t c[NB][1 << BK];
#pragma unroll
    for (int bl = 0; bl < NB; ++bl) {
      c[bl][0] = 0u;
#pragma unroll
      for (int m = 1; m < (1 << BK); ++m) {
        const int t = __builtin_ctz(m), k = BK * bl + t;
        const uint32_t xt = k < D ? xin[k] : 0u;
        c[bl][m] = (m & (m - 1)) ? (c[bl][m & (m - 1)] ^ xt) : xt;
      }
    }
    fr_outputs<D, P, NB, BK>(y, j, c, std::make_integer_sequence<int, P>{});
  }
}

// y = sum_k c_k * x_k over GF(2^8) with per-lane coefficients: Horner over the
// coefficient bits; bit b of c_k becomes a lane mask (v_bfe_i32) that enters
// the 4 dwords of the chunk through v_bitop3 y ^ (x & m).  The mask and its
// four uses are one asm unit: left to itself the compiler computes all 8*DMAX
// masks once, keeps them live to share across the 4 dwords, and runs out of
// VGPRs (124 -> 60 for DMAX = 10).
template <int POS>
__device__ __forceinline__ void mxor4(V4& y, const V4& x, uint32_t cw) {
  uint32_t m;
  asm("v_bfe_i32 %4, %5, %6, 1\n\t"
      "v_bitop3_b32 %0, %0, %7, %4 bitop3:0x78\n\t"
      "v_bitop3_b32 %1, %1, %8, %4 bitop3:0x78\n\t"
      "v_bitop3_b32 %2, %2, %9, %4 bitop3:0x78\n\t"
      "v_bitop3_b32 %3, %3, %10, %4 bitop3:0x78"
      : "+v"(y.v[0]), "+v"(y.v[1]), "+v"(y.v[2]), "+v"(y.v[3]), "=&v"(m)
      : "v"(cw), "i"(POS), "v"(x.v[0]), "v"(x.v[1]), "v"(x.v[2]), "v"(x.v[3]));
}

template <int DMAX, int B, int K>
__device__ __forceinline__ void hv_terms(V4& y, const V4* x, const uint32_t* cw) {
  mxor4<8 * (K & 3) + B>(y, x[K], cw[K >> 2]);
  if constexpr (K + 1 < DMAX) hv_terms<DMAX, B, K + 1>(y, x, cw);
}

template <int DMAX, int B>
__device__ __forceinline__ void hv_bits(V4& y, const V4* x, const uint32_t* cw) {
  if constexpr (B != 7) xt4(y);
  hv_terms<DMAX, B, 0>(y, x, cw);
  if constexpr (B > 0) hv_bits<DMAX, B - 1>(y, x, cw);
}

template <int DMAX>
__device__ __forceinline__ V4 horner_var(const V4* x, const uint32_t* cw) {
  V4 y{{0u, 0u, 0u, 0u}};
  hv_bits<DMAX, 7>(y, x, cw);
  return y;
}

__device__ __forceinline__ uint32_t ld32(const uint8_t* p) {
  return *reinterpret_cast<const uint32_t*>(p);
}

__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_amdgcn_perm(hi, lo, sel);
}

}  // namespace kern
}  // namespace ugo
