// fec_experiments.hpp -- encode / reconstruct kernels measured and not
// shipped, kept for the A/B harnesses that time them (tools/jvariants.hip:
// k_encode_fr; tools/qaprobe.hip: k_apply_ql).  Included after
// ugo_amd/csrc/fec_kernels.hip, whose helpers they use.  Not product code.
#pragma once

namespace ugo {
namespace kern {

// k_encode_g with the network in Four-Russians form (cparity_fr).  A/B only
// (tools/jvariants.hip): left to itself the scheduler builds all four dwords'
// tables at once (256 VGPRs + 46 AGPRs, 723-743 us); production runs
// k_encode_frs below.
template <int D, int P, int NTS = 0, int GR = D, int BS = 256, int LR = GR, int WPE = 1>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(WPE))) void k_encode_fr(Batch a) {
  static_assert(LR >= GR, "the stage holds at least the staged rows");
  __shared__ u32x4 stage[BS / 64][LR][64];
  const uint32_t item = blockIdx.x * BS + threadIdx.x;
  if (item >= a.items) return;
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const Loc l = locate(a, item);
#pragma unroll
  for (int k = 0; k < GR; ++k) lds_dma16(l.gp + static_cast<uint64_t>(k) * a.rstride, &stage[w][k][0]);
  V4 x[D];
#pragma unroll
  for (int k = GR; k < D; ++k) x[k] = load16<1>(l.gp + static_cast<uint64_t>(k) * a.rstride);
  lds_dma_wait();
#pragma unroll
  for (int k = 0; k < GR; ++k) x[k] = lds16(&stage[w][k][lane]);
  V4 y[P];
  cparity_fr<D, P>(y, x);
#pragma unroll
  for (int i = 0; i < P; ++i) store16<NTS>(l.gp + static_cast<uint64_t>(D + i) * a.rstride, y[i], l.nb);
}

// Wait until at most VM of the wave's vector-memory ops are outstanding, then
// read two staged input chunks (this lane's 16 B of two LDS slots) -- one asm
// unit, its outputs ready when it ends; `tok` orders it after the DMAs that
// filled the slots and the next DMAs after it.
template <int VM>
__device__ __forceinline__ void lds_pair(V4& x0, V4& x1, uint32_t ad0, uint32_t ad1, uint32_t& tok) {
  u32x4 v0, v1;
#define UGO_LDS_PAIR(N)                                                                              \
  asm("s_waitcnt vmcnt(" #N ")\n\tds_read_b128 %0, %3\n\tds_read_b128 %1, %4\n\ts_waitcnt lgkmcnt(0)" \
      : "=&v"(v0), "=&v"(v1), "+s"(tok)                                                             \
      : "v"(ad0), "v"(ad1))
  if constexpr (VM == 0) UGO_LDS_PAIR(0);
  else if constexpr (VM == 2) UGO_LDS_PAIR(2);
  else if constexpr (VM == 4) UGO_LDS_PAIR(4);
  else if constexpr (VM == 6) UGO_LDS_PAIR(6);
  else if constexpr (VM == 8) UGO_LDS_PAIR(8);
  else if constexpr (VM == 10) UGO_LDS_PAIR(10);
  else static_assert(VM == 0, "lds_pair: vmcnt 0..10, even");
#undef UGO_LDS_PAIR
  x0 = V4{{v0.x, v0.y, v0.z, v0.w}};
  x1 = V4{{v1.x, v1.y, v1.z, v1.w}};
}

// k_apply_qb with its inputs prefetched by LDS-DMA (A/B candidate, round 3):
// each wave keeps R input chunks in flight in an R-slot LDS ring instead of
// one pair in registers, without spending VGPRs on them.  The input loop is
// unrolled over R/2 pairs so every slot and every vmcnt is a constant; the
// last R/2 pairs drain the ring.  Needs d % R == 0 (the (32,8) jumbo code).
template <int EMAX, int MODE, int R = 8, bool UNROLL = true>
__global__ __launch_bounds__(256) void k_apply_ql(Batch a) {
  static_assert(R % 2 == 0 && R >= 4 && R <= 12, "ring of 4..12 slots");
  __shared__ u32x4 stage[4][R][64];
  const uint32_t cpad = (a.chunks + 63u) & ~63u;
  const uint32_t wfirst = blockIdx.x * 256u + (__builtin_amdgcn_readfirstlane(threadIdx.x) & ~63u);
  if (wfirst >= a.items) return;  // a.items = groups * cpad here
  const uint32_t gl = __builtin_amdgcn_readfirstlane(wfirst / cpad);
  const uint64_t g = a.g0 + gl;
  const uint64_t dU = rfl64(reinterpret_cast<uint64_t>(desc_for<MODE>(a, g)));
  auto dword = [&](uint32_t off) -> uint32_t { return *(ctab_t)(dU + off); };
  const uint32_t hA = dword(0);
  const uint32_t st = (hA >> 16) & 0xffu;
  const uint32_t e = st ? 0u : (a.data_only ? ((hA >> 8) & 0xffu) : (hA & 0xffu));
  const uint32_t c = blockIdx.x * 256u + threadIdx.x - gl * cpad;
  const bool live = c < a.chunks;
  const bool wst = MODE != 0 && a.status != nullptr && c == 0;
  if (e == 0) {  // wave-uniform
    if (wst) a.status[g] = static_cast<int8_t>(st);
    return;
  }
  const uint32_t coff = live ? c * 16u : 0u;
  const uint8_t* gbase = a.base + g * a.gstride;  // wave-uniform
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
  const uint32_t sbase = lds_addr(&stage[w][0][0]);     // wave-uniform: M0 of a slot's DMA
  const uint32_t lbase = lds_addr(&stage[w][0][lane]);  // this lane's 16 B of slot 0
  uint32_t tok = 0;
  auto dma = [&](uint32_t k, uint32_t slot) {  // input k into a slot
    const uint32_t r = (dword(4 + (k & ~3u)) >> (8 * (k & 3u))) & 0xffu;
    uint32_t co = coff;
    asm("" : "+v"(co));
    lds_dma16_nt_asm(gbase + static_cast<uint64_t>(r) * a.rstride + co, sbase + 1024u * slot, tok);
  };
  const uint32_t cbase = 4 + a.dpad + a.epad;
  V4 acc[EMAX];
#pragma unroll
  for (int i = 0; i < EMAX; ++i) acc[i] = V4{{0u, 0u, 0u, 0u}};
  auto fold = [&](uint32_t k, const V4& x0, const V4& x1) {  // inputs k, k+1 (k even)
    uint32_t s0[4], s1[4], s2[4], r0[4], r1[4], r2[4];
    p_sel(x0, s0, s1, s2);
    p_sel(x1, r0, r1, r2);
#pragma unroll
    for (int i = 0; i < EMAX; ++i) {
      if (i >= static_cast<int>(e)) continue;
      const uint32_t off = cbase + i * a.dpad + (k & ~3u);
      uint32_t t[5], u[5];
      {
        const ctab_t tA = (ctab_t)(a.mult) + 8u * ((dword(off) >> (8 * (k & 3u))) & 0xffu);
#pragma unroll
        for (int q = 0; q < 5; ++q) t[q] = tA[q];
      }
      {
        const ctab_t tB = (ctab_t)(a.mult) + 8u * ((dword(off) >> (8 * ((k + 1) & 3u))) & 0xffu);
#pragma unroll
        for (int q = 0; q < 5; ++q) u[q] = tB[q];
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t y = xor3(acc[i].v[q], perm(t[1], t[0], s0[q]), perm(t[3], t[2], s1[q]));
        y = xor3(y, perm(0u, t[4], s2[q]), perm(u[1], u[0], r0[q]));
        acc[i].v[q] = xor3(y, perm(u[3], u[2], r1[q]), perm(0u, u[4], r2[q]));
      }
    }
  };
#pragma unroll
  for (int j = 0; j < R; ++j) dma(j, j);  // prime the ring
  uint32_t k0 = 0;
  if constexpr (UNROLL) {
    for (; k0 + R < a.d; k0 += R) {  // steady state: a pair read, its slots refilled R inputs ahead
#pragma unroll
      for (int j = 0; j < R; j += 2) {
        V4 x0, x1;
        lds_pair<R - 2>(x0, x1, lbase + 1024u * j, lbase + 1024u * (j + 1), tok);
        dma(k0 + R + j, j);
        dma(k0 + R + j + 1, j + 1);
        fold(k0 + j, x0, x1);
      }
    }
  } else {
    // one pair per iteration, slots at run time (R a power of two), and one
    // copy of the fold: the drain waits for all its inputs at once
    static_assert((R & (R - 1)) == 0, "R a power of two");
    for (uint32_t k = 0; k < a.d; k += 2) {
      const uint32_t sl = k & (R - 1);
      V4 x0, x1;
      const bool refill = k + R < a.d;  // wave-uniform
      if (!refill) asm volatile("s_waitcnt vmcnt(0)" : "+s"(tok));
      lds_pair<R - 2>(x0, x1, lbase + 1024u * sl, lbase + 1024u * (sl + 1), tok);
      if (refill) {
        dma(k + R, sl);
        dma(k + R + 1, sl + 1);
      }
      fold(k, x0, x1);
    }
    k0 = a.d;  // nothing left for the drain below
  }
  // drain: the last R inputs, nothing refilled (VM = inputs still in flight after this pair)
#define UGO_DRAIN(J)                                                                        \
  if constexpr (UNROLL && J < R) {                                                          \
    V4 x0, x1;                                                                              \
    lds_pair<(R - J - 2 > 0 ? R - J - 2 : 0)>(x0, x1, lbase + 1024u * J, lbase + 1024u * (J + 1), tok); \
    fold(k0 + J, x0, x1);                                                                   \
  }
  UGO_DRAIN(0) UGO_DRAIN(2) UGO_DRAIN(4) UGO_DRAIN(6) UGO_DRAIN(8) UGO_DRAIN(10)
#undef UGO_DRAIN
  if (live) {
    const uint32_t nb = a.S - coff;
    constexpr int NO = (EMAX + 3) / 4;
    uint32_t orw[NO];
#pragma unroll
    for (int q = 0; q < NO; ++q) orw[q] = dword(4 + a.dpad + 4 * q);
    uint8_t* gp = const_cast<uint8_t*>(gbase) + coff;
#pragma unroll
    for (int i = 0; i < EMAX; ++i) {
      if (i >= static_cast<int>(e)) continue;
      const uint32_t r = (orw[i >> 2] >> (8 * (i & 3))) & 0xffu;
      store16<2>(out_row(a, gp, g, coff, r, i), acc[i], nb);
    }
  }
  if (wst) a.status[g] = 0;
}

}  // namespace kern
}  // namespace ugo
