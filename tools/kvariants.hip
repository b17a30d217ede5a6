// kvariants.hip -- interleaved A/B timing of kernel variants (one process,
// N rounds x M variants, median reported: cdna_hip_programming.md §5.4 rule 24).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/kvariants tools/kvariants.hip
// Not product code: it includes the kernel TU to instantiate variants.
#include "../ugo_amd/csrc/fec_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <string>
#include <vector>

using namespace ugo;
using namespace ugo::kern;

#include "ab_common.hpp"

// Memory-pattern ceiling of the reconstruct: the wave-scalar descriptor
// prologue, survivor loads and erased-row stores of k_apply_p, with the GF
// arithmetic replaced by a plain XOR of the survivors (wrong values, same bytes).
// OOP (probe): erased row i goes to output slot i of a separate planar batch
// [4][G][pitch] at a.status (reused as a byte pointer), not back in place.
template <int NT, bool GL = false, bool OOP = false>
__global__ __launch_bounds__(256) void k_pattern_rec(Batch a) {
  __shared__ u32x4 stage[GL ? 4 : 1][GL ? 10 : 1][64];
  const uint32_t wfirst = blockIdx.x * 256u + (__builtin_amdgcn_readfirstlane(threadIdx.x) & ~63u);
  const uint32_t item = blockIdx.x * 256u + threadIdx.x;
  if (wfirst >= a.items) return;
  const uint32_t wlast = min(wfirst + 63u, a.items - 1u);
  const uint32_t gA = wfirst / a.chunks, gB = wlast / a.chunks;
  const uint8_t* dA = desc_for<1>(a, a.g0 + gA);
  const uint8_t* dB = desc_for<1>(a, a.g0 + gB);
  const uint32_t hA = ld32(dA), hB = ld32(dB);
  uint32_t rA[3], rB[3];
  for (int w = 0; w < 3; ++w) { rA[w] = ld32(dA + 4 + 4 * w); rB[w] = ld32(dB + 4 + 4 * w); }
  const uint32_t oA = ld32(dA + 4 + a.dpad), oB = ld32(dB + 4 + a.dpad);
  if (item >= a.items) return;
  const uint32_t gl = item / a.chunks;
  const bool inB = gl != gA;
  const uint32_t c = item - gl * a.chunks;
  const uint32_t e = (inB ? hB : hA) & 0xffu;
  uint8_t* gp = a.base + (a.g0 + gl) * a.gstride + static_cast<uint64_t>(c) * 16u;
  const uint32_t nb = a.S - c * 16u;
  V4 y{{0u, 0u, 0u, 0u}};
  if constexpr (GL) {
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      const uint32_t rw = inB ? rB[k >> 2] : rA[k >> 2];
      const uint32_t r = (rw >> (8 * (k & 3))) & 0xffu;
      lds_dma16(gp + static_cast<uint64_t>(r) * a.rstride, &stage[w][k][0]);
    }
    lds_dma_wait();
#pragma unroll
    for (int k = 0; k < 10; ++k) xor4(y, lds16(&stage[w][k][lane]));
  } else {
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      const uint32_t rw = inB ? rB[k >> 2] : rA[k >> 2];
      const uint32_t r = (rw >> (8 * (k & 3))) & 0xffu;
      xor4(y, load16<NT>(gp + static_cast<uint64_t>(r) * a.rstride));
    }
  }
  const uint32_t orows = inB ? oB : oA;
  for (int i = 0; i < 4; ++i) {
    if (i >= static_cast<int>(e)) continue;
    const uint32_t r = (orows >> (8 * i)) & 0xffu;
    y.v[0] += i;
    if constexpr (OOP)
      store16<NT>(reinterpret_cast<uint8_t*>(a.status) + static_cast<uint64_t>(i) * a.rstride +
                      (a.g0 + gl) * a.gstride + static_cast<uint64_t>(c) * 16u, y, nb);
    else
      store16<NT>(gp + static_cast<uint64_t>(r) * a.rstride, y, nb);
  }
}

// Memory-pattern probes for the random-erasure reconstruct: READS 0 = the
// first 10 present rows (the real survivor set), 1 = every present row (11 of
// 13: no read gaps), 2 = all 13 rows; then the erased rows are written.
template <int READS>
__global__ __launch_bounds__(256) void k_pattern_probe(Batch a) {
  const uint32_t item = blockIdx.x * 256u + threadIdx.x;
  if (item >= a.items) return;
  const uint32_t gl = item / a.chunks;
  const uint32_t c = item - gl * a.chunks;
  const uint64_t m = a.present[a.g0 + gl];
  uint8_t* gp = a.base + (a.g0 + gl) * a.gstride + static_cast<uint64_t>(c) * 16u;
  V4 y{{0u, 0u, 0u, 0u}};
  int taken = 0;
#pragma unroll
  for (int r = 0; r < 13; ++r) {
    const bool pres = (m >> r) & 1u;
    const bool rd = READS == 2 ? true : (READS == 1 ? pres : (pres && taken < 10));
    taken += pres;
    if (rd) xor4(y, load16<1>(gp + static_cast<uint64_t>(r) * a.rstride));
  }
#pragma unroll
  for (int r = 0; r < 13; ++r)
    if (!((m >> r) & 1u)) { y.v[0] += r; store16<0>(gp + static_cast<uint64_t>(r) * a.rstride, y, 16); }
}

// Compute-free encode pattern: the 10 data rows in (GR of them by LDS-DMA nt,
// the rest nt register loads), 3 XOR "parity" rows out.
template <int GR, int NTS>
__global__ __launch_bounds__(256) void k_pattern_enc(Batch a) {
  __shared__ u32x4 stage[4][GR ? GR : 1][64];
  const uint32_t item = blockIdx.x * 256u + threadIdx.x;
  if (item >= a.items) return;
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const Loc l = locate(a, item);
  V4 x[10];
#pragma unroll
  for (int k = 0; k < GR; ++k) lds_dma16(l.gp + static_cast<uint64_t>(k) * a.rstride, &stage[w][k][0]);
#pragma unroll
  for (int k = GR; k < 10; ++k) x[k] = load16<1>(l.gp + static_cast<uint64_t>(k) * a.rstride);
  if constexpr (GR > 0) {
    lds_dma_wait();
#pragma unroll
    for (int k = 0; k < GR; ++k) x[k] = lds16(&stage[w][k][lane]);
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    V4 y = x[i];
#pragma unroll
    for (int k = 3; k < 10; ++k)
      if ((k + i) & 1) xor4(y, x[k]);
    store16<NTS>(l.gp + static_cast<uint64_t>(10 + i) * a.rstride, y, 16);
  }
}

// Persistent, pipelined k_encode_g (A/B only): a wave walks 64-item steps at a
// grid stride; once step t's rows are in registers, step t+1's row loads are
// issued into the same stage, streaming while step t is computed and stored.
template <int D, int P, int NTS, int GR>
__global__ __launch_bounds__(256) void k_encode_gp(Batch a) {
  __shared__ u32x4 stage[4][GR][64];
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t nsteps = (a.items + 63u) / 64u, stride = gridDim.x * 4u;
  uint32_t step = blockIdx.x * 4u + w;
  if (step >= nsteps) return;
  uint32_t item = step * 64u + lane;
  Loc l = locate(a, min(item, a.items - 1u));
  V4 x[D];
#pragma unroll
  for (int k = 0; k < GR; ++k) lds_dma16(l.gp + static_cast<uint64_t>(k) * a.rstride, &stage[w][k][0]);
#pragma unroll
  for (int k = GR; k < D; ++k) x[k] = load16<1>(l.gp + static_cast<uint64_t>(k) * a.rstride);
  for (;;) {
    lds_dma_wait();
#pragma unroll
    for (int k = 0; k < GR; ++k) x[k] = lds16(&stage[w][k][lane]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    V4 xc[D];
#pragma unroll
    for (int k = 0; k < D; ++k) xc[k] = x[k];
    const uint32_t cur = item;
    const Loc lc = l;
    step += stride;
    const bool more = step < nsteps;
    if (more) {
      item = step * 64u + lane;
      l = locate(a, min(item, a.items - 1u));
#pragma unroll
      for (int k = 0; k < GR; ++k) lds_dma16(l.gp + static_cast<uint64_t>(k) * a.rstride, &stage[w][k][0]);
#pragma unroll
      for (int k = GR; k < D; ++k) x[k] = load16<1>(l.gp + static_cast<uint64_t>(k) * a.rstride);
    }
    if (cur < a.items) cparity_store<D, P, NTS>(lc.gp, a.rstride, lc.nb, xc, std::make_integer_sequence<int, P>{});
    if (!more) break;
  }
}

// Encode with CPT chunks per lane, wave-contiguous: lane l of wave w takes
// chunks 64*CPT*w + 64*j + l (j < CPT), so each wave covers CPT KiB of every
// row (A/B: does per-wave contiguity beyond 1 KiB help the cold pattern?).
template <int CPT, int NT, int GR = 0>
__global__ __launch_bounds__(256) void k_encode_cpt(Batch a) {
  __shared__ u32x4 stage[GR ? 4 : 1][GR ? GR : 1][CPT][64];
  const uint32_t wave = (blockIdx.x * 256u + threadIdx.x) >> 6, lane = threadIdx.x & 63u;
  const uint32_t w = threadIdx.x >> 6;
  V4 x[CPT][10];
  Loc l[CPT];
  bool ok[CPT];
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    const uint32_t item = wave * 64u * CPT + 64u * j + lane;
    ok[j] = item < a.items;
    l[j] = locate(a, ok[j] ? item : 0u);
    if (ok[j]) {
#pragma unroll
      for (int k = 0; k < GR; ++k) lds_dma16(l[j].gp + static_cast<uint64_t>(k) * a.rstride, &stage[w][k][j][0]);
#pragma unroll
      for (int k = GR; k < 10; ++k) x[j][k] = load16<NT>(l[j].gp + static_cast<uint64_t>(k) * a.rstride);
    }
  }
  if constexpr (GR > 0) {
    lds_dma_wait();
#pragma unroll
    for (int j = 0; j < CPT; ++j)
#pragma unroll
      for (int k = 0; k < GR; ++k) x[j][k] = lds16(&stage[w][k][j][lane]);
  }
#pragma unroll
  for (int j = 0; j < CPT; ++j)
    if (ok[j]) cparity_store<10, 3, NT>(l[j].gp, a.rstride, l[j].nb, x[j], std::make_integer_sequence<int, 3>{});
}

// Store cache-policy probe (A/B TIMING only): k_encode_g's loads, parity stored
// with global_store_dwordx4 and the given cache modifiers (always whole 16 B:
// the (10,3) pitch 1360 leaves room past the last chunk).  Inline-asm VMEM
// stores are invisible to the compiler's hazard tracking, so the data VGPRs can
// be reused before the store reads them: the VALUES are not trustworthy (the
// same store in k_encode_g failed the bit-exact check), only the timing is.
template <int POL>
__device__ __forceinline__ void store_pol(uint8_t* p, const V4& y) {
  const u32x4 v = {y.v[0], y.v[1], y.v[2], y.v[3]};
  if constexpr (POL == 0) asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(p), "v"(v) : "memory");
  if constexpr (POL == 1) asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(p), "v"(v) : "memory");
  if constexpr (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  if constexpr (POL == 3) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
  if constexpr (POL == 4) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
  if constexpr (POL == 5) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
  if constexpr (POL == 6) asm volatile("global_store_dwordx4 %0, %1, off sc0" ::"v"(p), "v"(v) : "memory");
  if constexpr (POL == 7) asm volatile("global_store_dwordx4 %0, %1, off sc0 nt" ::"v"(p), "v"(v) : "memory");
}

template <int POL>
__global__ __launch_bounds__(256) void k_encode_pol(Batch a) {
  __shared__ u32x4 stage[4][8][64];
  const uint32_t item = blockIdx.x * 256u + threadIdx.x;
  if (item >= a.items) return;
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const Loc l = locate(a, item);
#pragma unroll
  for (int k = 0; k < 8; ++k) lds_dma16(l.gp + static_cast<uint64_t>(k) * a.rstride, &stage[w][k][0]);
  V4 x[10];
#pragma unroll
  for (int k = 8; k < 10; ++k) x[k] = load16<1>(l.gp + static_cast<uint64_t>(k) * a.rstride);
  lds_dma_wait();
#pragma unroll
  for (int k = 0; k < 8; ++k) x[k] = lds16(&stage[w][k][lane]);
  store_pol<POL>(l.gp + 10 * a.rstride, cparity<10, 3, 0>(x));
  store_pol<POL>(l.gp + 11 * a.rstride, cparity<10, 3, 1>(x));
  store_pol<POL>(l.gp + 12 * a.rstride, cparity<10, 3, 2>(x));
}

__global__ __launch_bounds__(256) void k_flush_read(const u32x4* __restrict__ a, uint32_t* out, uint64_t n16) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i >= n16) return;
  const u32x4 v = a[i];
  if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9e3779b9u) out[0] = v.x;
}

// Layout probe (A/B only): compute-free encode pattern over a TILED planar
// layout [G/T][13][T][pitch] -- each tile of T groups is planar, tiles follow
// each other -- instead of one planar [13][G][pitch].
template <int T>
__global__ __launch_bounds__(256) void k_pattern_tiled(Batch a) {
  const uint32_t item = blockIdx.x * 256u + threadIdx.x;
  if (item >= a.items) return;
  const uint32_t g = item / a.chunks, c = item - g * a.chunks;
  const uint64_t tile = g / T, gi = g % T;
  const uint64_t rs = static_cast<uint64_t>(T) * a.gstride;  // row stride inside a tile
  uint8_t* gp = a.base + tile * 13ull * rs + gi * a.gstride + c * 16ull;
  V4 x[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) x[k] = load16<1>(gp + k * rs);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    V4 y = x[i];
#pragma unroll
    for (int k = 3; k < 10; ++k)
      if ((k + i) & 1) xor4(y, x[k]);
    store16<2>(gp + (10 + i) * rs, y, 16);
  }
}

// Cold-regime ceilings: write-only and copy streams over a whole batch buffer.
template <int NTS>
__global__ __launch_bounds__(256) void k_write_stream(Batch a, uint64_t n16) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i >= n16) return;
  const u32x4 v = {static_cast<uint32_t>(i), 1u, 2u, 3u};
  u32x4* q = reinterpret_cast<u32x4*>(a.base) + i;
  if constexpr (NTS) __builtin_nontemporal_store(v, q); else *q = v;
}
template <int NTS>
__global__ __launch_bounds__(256) void k_copy_stream(Batch a, uint64_t n16) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i >= n16) return;
  const u32x4* src = reinterpret_cast<const u32x4*>(a.base) + i;
  u32x4* dst = reinterpret_cast<u32x4*>(a.base) + n16 + i;
  const u32x4 v = __builtin_nontemporal_load(src);
  if constexpr (NTS) __builtin_nontemporal_store(v, dst); else *dst = v;
}

int main(int argc, char** argv) {
  const int d = 10, p = 3, n = 13;
  const uint32_t S = 1350, pitch = 1360;
  const uint64_t G = argc > 1 ? atoll(argv[1]) : 65536;
  const int rounds = argc > 2 ? atoi(argv[2]) : 15;
  uint8_t* buf;
  uint64_t* masks;
  CK(hipMalloc(&buf, G * n * pitch));
  CK(hipMalloc(&masks, G * 8));
  std::vector<uint8_t> h(G * n * pitch);
  uint64_t st = 0x5EED;
  for (auto& b : h) { st = st * 6364136223846793005ull + 1442695040888963407ull; b = st >> 56; }
  CK(hipMemcpy(buf, h.data(), h.size(), hipMemcpyHostToDevice));
  std::vector<uint64_t> hm(G);
  for (uint64_t g = 0; g < G; ++g) {
    st = st * 6364136223846793005ull + 1442695040888963407ull;
    int a = (st >> 33) % n, b = (a + 1 + (st >> 40) % (n - 1)) % n;
    hm[g] = ((1ull << n) - 1) & ~(1ull << a) & ~(1ull << b);
  }
  CK(hipMemcpy(masks, hm.data(), G * 8, hipMemcpyHostToDevice));
  const uint32_t dpad = 12, epad = 4, stride = 64;
  std::vector<uint8_t> tab;
  build_table(d, p, dpad, epad, stride, tab);
  uint8_t* dtab;
  CK(hipMalloc(&dtab, tab.size()));
  CK(hipMemcpy(dtab, tab.data(), tab.size(), hipMemcpyHostToDevice));
  std::vector<uint8_t> tabc;
  build_table(d, p, dpad, epad, stride, tabc, true);
  uint8_t* dtabc;
  CK(hipMalloc(&dtabc, tabc.size()));
  CK(hipMemcpy(dtabc, tabc.data(), tabc.size(), hipMemcpyHostToDevice));

  std::vector<uint8_t> hmul(256 * 32);
  ugo::gf::perm_tables(hmul.data());
  uint32_t* dmul;
  CK(hipMalloc(&dmul, hmul.size()));
  CK(hipMemcpy(dmul, hmul.data(), hmul.size(), hipMemcpyHostToDevice));
  Batch a{};
  a.mult = dmul;
  a.base = buf; a.gstride = n * pitch; a.rstride = pitch; a.nmask = (1ull << n) - 1; a.S = S;
  a.chunks = 85; a.items = G * 85; a.desc = dtab; a.present = masks; a.desc_stride = stride; a.d = d;
  a.dpad = dpad; a.epad = epad;
  Batch pl = a;  // planar [13][G][pitch]
  pl.gstride = pitch;
  pl.rstride = G * pitch;
  const double enc_bytes = double(G) * n * S, dec_bytes = double(G) * 12 * S;

  struct Var { std::string name; double bytes; std::function<void()> go; std::vector<float> t; };
  std::vector<Var> vars;
  auto add = [&](auto kern, const Batch& b, double bytes, std::string nm) {
    const uint32_t grid = (b.items + 255) / 256;
    vars.push_back({nm, bytes, [=]() { hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, b); }, {}});
  };
  // same erasure pattern (rows 3 and 11) for every group: isolates the cost of
  // per-group scattered survivor/erased rows from the arithmetic
  uint64_t* masks_fixed;
  CK(hipMalloc(&masks_fixed, G * 8));
  std::vector<uint64_t> hf(G, ((1ull << n) - 1) & ~(1ull << 3) & ~(1ull << 11));
  CK(hipMemcpy(masks_fixed, hf.data(), G * 8, hipMemcpyHostToDevice));
  for (int lay = 1; lay < 2; ++lay) {  // 0 = interleaved: see profiles/r1/kvariants_interleaved_ab.jsonl
    const Batch& b = lay ? pl : a;
    const std::string L = lay ? "planar" : "interl";
    add(k_encode_c<10, 3, 0>, b, enc_bytes, "enc " + L + " nt0");
    add(k_encode_c<10, 3, 1>, b, enc_bytes, "enc " + L + " nt1");
    add(k_encode_c<10, 3, 1, 1>, b, enc_bytes, "enc " + L + " nt1 xcd-contiguous");
    add(k_encode_c<10, 3, 3>, b, enc_bytes, "enc " + L + " nt3");
    add(k_apply<10, 1, 0>, b, dec_bytes, "dec " + L + " nt0");
    add(k_apply<10, 1, 1>, b, dec_bytes, "dec " + L + " nt1");
    add(k_apply<10, 1, 3>, b, dec_bytes, "dec " + L + " nt3");
    {
      Batch b1 = b;
      b1.pass = (b.items + 63u) / 64u * 64u;
      add(k_apply_w<10, 1, 3, 1>, b1, dec_bytes, "dec " + L + " nt3 wave-scalar-desc cpt1");
    }
    add(k_apply_p<10, 1, 1, 1>, b, dec_bytes, "dec " + L + " nt1 perm-tables scalar-pick");
    add(k_apply_p<10, 1, 1, 1, 1, 4, true, 1>, b, dec_bytes, "dec " + L + " nt1 perm-tables xcd-contiguous");
    add(k_apply_p<10, 1, 1, 1, 1, 3, true>, b, dec_bytes, "dec " + L + " nt1 perm pair emax3");
    add(k_apply_p<10, 1, 1, 1, 1, 3, false>, b, dec_bytes, "dec " + L + " nt1 perm single emax3");
    add(k_pattern_rec<1>, b, dec_bytes, "dec " + L + " MEMORY PATTERN ONLY nt1 (xor, no GF)");
    add(k_pattern_rec<3>, b, dec_bytes, "dec " + L + " MEMORY PATTERN ONLY nt3 (xor, no GF)");
    add(k_apply_p<12, 1, 1>, b, dec_bytes, "dec " + L + " nt1 perm-tables dmax12");
    Batch bf = b;
    bf.present = masks_fixed;
    add(k_apply<10, 1, 3>, bf, dec_bytes, "dec " + L + " nt3 fixed-pattern");
    // same fixed pattern through a uniform (MODE 0) descriptor: no per-lane
    // mask -> descriptor dependent loads, scalar descriptor reads
    Batch bu = b;
    bu.desc = dtab + hf[0] * stride;
    add(k_apply<10, 0, 3>, bu, dec_bytes, "dec " + L + " nt3 fixed-pattern uniform-desc");
    // fixed pattern: every wave takes k_apply_p's uniform path (dA == dB, no
    // per-lane table pick); against the compute-free pattern of the same rows
    add(k_apply_p<10, 1, 1>, bf, dec_bytes, "dec " + L + " perm nt1 fixed-pattern (no picks)");
    add(k_apply_p<10, 1, 1, 1, 1, 4, true, 0, 10>, bf, dec_bytes, "dec " + L + " perm lds-dma fixed-pattern (no picks)");
    add(k_pattern_rec<1>, bf, dec_bytes, "dec " + L + " MEMORY PATTERN ONLY nt1 fixed-pattern");
    add(k_pattern_rec<1, true>, bf, dec_bytes, "dec " + L + " MEMORY PATTERN ONLY lds-dma fixed-pattern");
    add(k_pattern_probe<0>, b, dec_bytes, "dec " + L + " PROBE read first-10-present, write erased");
    add(k_pattern_probe<1>, b, dec_bytes, "dec " + L + " PROBE read all 11 present, write erased");
    add(k_pattern_probe<2>, b, dec_bytes, "dec " + L + " PROBE read all 13, write erased");
    add(k_pattern_probe<0>, bf, dec_bytes, "dec " + L + " PROBE fixed-pattern first-10");
    add(k_pattern_probe<1>, bf, dec_bytes, "dec " + L + " PROBE fixed-pattern all 11 present");
  }

  // encode -> reconstruct back-to-back (the bench step): the encode's store
  // policy changes what the following reconstruct finds in L2 / MALL
  auto pair = [&](auto ke, auto kd, const Batch& b, std::string nm) {
    const uint32_t grid = (b.items + 255) / 256;
    vars.push_back({nm, enc_bytes + dec_bytes, [=]() {
      hipLaunchKernelGGL(ke, dim3(grid), dim3(256), 0, 0, b);
      hipLaunchKernelGGL(kd, dim3(grid), dim3(256), 0, 0, b);
    }, {}});
  };
  pair(k_encode_c<10, 3, 1>, k_apply_p<10, 1, 1>, pl, "pair planar enc-nt1 perm-nt1");
  pair(k_encode_c<10, 3, 1, 1>, k_apply_p<10, 1, 1, 1, 1, 4, true, 1>, pl, "pair planar enc-nt1 perm-nt1 xcd-contiguous");
  pair(k_encode_c<10, 3, 3>, k_apply_p<10, 1, 1>, pl, "pair planar enc-nt3 perm-nt1");
  pair(k_encode_c<10, 3, 1>, k_apply_p<10, 1, 3>, pl, "pair planar enc-nt1 perm-nt3");
  pair(k_encode_c<10, 3, 3>, k_apply_p<10, 1, 3>, pl, "pair planar enc-nt3 perm-nt3");
  pair(k_encode_c<10, 3, 1>, k_apply_p<10, 1, 0>, pl, "pair planar enc-nt1 perm-nt0");
  // Cold-HBM regime (argv[3] == "cold"): every launch works on the next of 4
  // independent batches, so no launch finds its batch's lines in the 256-MB
  // Infinity Cache.  Only these variants run in that mode.
  const bool cold = argc > 3 && std::string(argv[3]) == "cold";
  if (cold) {
    vars.clear();
    std::vector<Batch> rot(4, pl);
    for (int r = 1; r < 4; ++r) {
      uint8_t* nb;
      CK(hipMalloc(&nb, G * n * pitch));
      CK(hipMemcpy(nb, buf, G * n * pitch, hipMemcpyDeviceToDevice));
      rot[r].base = nb;
    }
    auto cnt = std::make_shared<int>(0);
    auto addr = [&](auto kern, double bytes, std::string nm) {
      const uint32_t grid = (pl.items + 255) / 256;
      vars.push_back({nm, bytes, [=]() { hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, rot[(*cnt)++ & 3]); }, {}});
    };
    auto pairr = [&](auto ke, auto kd, std::string nm) {
      const uint32_t grid = (pl.items + 255) / 256;
      vars.push_back({nm, enc_bytes + dec_bytes, [=]() {
        const Batch& b = rot[(*cnt)++ & 3];
        hipLaunchKernelGGL(ke, dim3(grid), dim3(256), 0, 0, b);
        hipLaunchKernelGGL(kd, dim3(grid), dim3(256), 0, 0, b);
      }, {}});
    };
    addr(k_encode_g<10, 3, 0, 8>, enc_bytes, "COLD enc lds-dma 8");
    addr(k_encode_g<10, 3, 2, 8>, enc_bytes, "COLD enc lds-dma 8, nt stores (production)");
    addr(k_pattern_tiled<512>, enc_bytes, "COLD enc PATTERN tiled planar T=512");
    addr(k_pattern_tiled<4096>, enc_bytes, "COLD enc PATTERN tiled planar T=4096");
    addr(k_pattern_tiled<16384>, enc_bytes, "COLD enc PATTERN tiled planar T=16384");
    addr(k_pattern_tiled<65536>, enc_bytes, "COLD enc PATTERN tiled planar T=65536 (= planar)");
    addr(k_encode_pol<0>, enc_bytes, "COLD enc POL store (plain)");
    addr(k_encode_pol<1>, enc_bytes, "COLD enc POL store nt");
    addr(k_encode_pol<2>, enc_bytes, "COLD enc POL store sc1");
    addr(k_encode_pol<3>, enc_bytes, "COLD enc POL store sc0 sc1");
    addr(k_encode_pol<4>, enc_bytes, "COLD enc POL store sc1 nt");
    addr(k_encode_pol<5>, enc_bytes, "COLD enc POL store sc0 sc1 nt");
    addr(k_encode_pol<6>, enc_bytes, "COLD enc POL store sc0");
    addr(k_encode_pol<7>, enc_bytes, "COLD enc POL store sc0 nt");
    addr(k_encode_g<10, 3, 0, 10>, enc_bytes, "COLD enc lds-dma 10");
    addr(k_encode_g<10, 3, 2, 10>, enc_bytes, "COLD enc lds-dma 10, nt stores");
    addr(k_encode_c<10, 3, 1>, enc_bytes, "COLD enc nt1");
    addr(k_encode_c<10, 3, 3>, enc_bytes, "COLD enc nt3");
    {
      const uint32_t g2 = (pl.items + 511) / 512, g4 = (pl.items + 1023) / 1024;
      vars.push_back({"COLD enc nt3, 2 chunks per lane (2 KiB per wave per row)", enc_bytes, [=]() {
        hipLaunchKernelGGL((k_encode_cpt<2, 3>), dim3(g2), dim3(256), 0, 0, rot[(*cnt)++ & 3]); }, {}});
      const uint32_t g3 = (pl.items + 767) / 768;
      vars.push_back({"COLD enc nt3, 3 chunks per lane", enc_bytes, [=]() {
        hipLaunchKernelGGL((k_encode_cpt<3, 3>), dim3(g3), dim3(256), 0, 0, rot[(*cnt)++ & 3]); }, {}});
      vars.push_back({"COLD enc nt3, 2 chunks per lane, 4 rows by LDS-DMA", enc_bytes, [=]() {
        hipLaunchKernelGGL((k_encode_cpt<2, 3, 4>), dim3(g2), dim3(256), 0, 0, rot[(*cnt)++ & 3]); }, {}});
      vars.push_back({"COLD enc nt3, 2 chunks per lane, 2 rows by LDS-DMA", enc_bytes, [=]() {
        hipLaunchKernelGGL((k_encode_cpt<2, 3, 2>), dim3(g2), dim3(256), 0, 0, rot[(*cnt)++ & 3]); }, {}});
      vars.push_back({"COLD enc nt1, 2 chunks per lane", enc_bytes, [=]() {
        hipLaunchKernelGGL((k_encode_cpt<2, 1>), dim3(g2), dim3(256), 0, 0, rot[(*cnt)++ & 3]); }, {}});
    }
    addr(k_encode_c<10, 3, 0>, enc_bytes, "COLD enc nt0");
    addr(k_apply_p<10, 1, 1>, dec_bytes, "COLD dec perm nt1");
    addr(k_apply_p<10, 1, 3>, dec_bytes, "COLD dec perm nt3 (production)");
    addr(k_apply_p<10, 1, 3, 0>, dec_bytes, "COLD dec perm nt3 TSEL0 (probe: no per-lane pick, B lanes wrong)");
    vars.push_back({"COLD pair enc nt3 2-chunk + dec nt3 reg", enc_bytes + dec_bytes, [=]() {
      const Batch& b = rot[(*cnt)++ & 3];
      hipLaunchKernelGGL((k_encode_cpt<2, 3>), dim3((pl.items + 511) / 512), dim3(256), 0, 0, b);
      hipLaunchKernelGGL((k_apply_p<10, 1, 3>), dim3((pl.items + 255) / 256), dim3(256), 0, 0, b); }, {}});
    addr(k_apply_p<10, 1, 3, 1, 1, 3>, dec_bytes, "COLD dec perm nt3 emax3");
    addr(k_apply_p<10, 1, 3, 1, 1, 4, false>, dec_bytes, "COLD dec perm nt3 unpaired");
    addr(k_apply_p<10, 1, 0>, dec_bytes, "COLD dec perm nt0");
    addr(k_apply_p<10, 1, 2>, dec_bytes, "COLD dec perm nt stores only");
    addr(k_apply_p<10, 1, 3, 1, 1, 4, true, 0, 10>, dec_bytes, "COLD dec perm lds-dma, nt stores");
    addr(k_apply_p<10, 1, 1, 1, 1, 4, true, 0, 10>, dec_bytes, "COLD dec perm lds-dma");
    addr(k_pattern_rec<3>, dec_bytes, "COLD dec MEMORY PATTERN ONLY nt3");
    addr(k_pattern_rec<3, true>, dec_bytes, "COLD dec MEMORY PATTERN ONLY lds-dma, nt stores");
    addr(k_apply_p<10, 1, 3, 1, 1, 3, true, 0, 10>, dec_bytes, "COLD dec perm lds-dma, nt stores, emax3");
    addr(k_apply_p<10, 1, 3, 1, 1, 4, true, 0, 8>, dec_bytes, "COLD dec perm lds-dma 8, nt stores");
    {
      const uint64_t bytes = G * n * pitch, n16w = bytes / 16, n16c = bytes / 32;
      vars.push_back({"COLD CEILING write-only stream nt", double(bytes), [=]() {
        hipLaunchKernelGGL(k_write_stream<1>, dim3((n16w + 255) / 256), dim3(256), 0, 0, rot[(*cnt)++ & 3], n16w); }, {}});
      vars.push_back({"COLD CEILING write-only stream plain", double(bytes), [=]() {
        hipLaunchKernelGGL(k_write_stream<0>, dim3((n16w + 255) / 256), dim3(256), 0, 0, rot[(*cnt)++ & 3], n16w); }, {}});
      vars.push_back({"COLD CEILING copy (half buffer -> other half) nt", double(bytes), [=]() {
        hipLaunchKernelGGL(k_copy_stream<1>, dim3((n16c + 255) / 256), dim3(256), 0, 0, rot[(*cnt)++ & 3], n16c); }, {}});
      vars.push_back({"COLD CEILING copy (half buffer -> other half) nt loads, plain stores", double(bytes), [=]() {
        hipLaunchKernelGGL(k_copy_stream<0>, dim3((n16c + 255) / 256), dim3(256), 0, 0, rot[(*cnt)++ & 3], n16c); }, {}});
    }
    addr(k_pattern_enc<0, 2>, enc_bytes, "COLD enc MEMORY PATTERN ONLY nt loads+stores");
    addr(k_pattern_enc<8, 2>, enc_bytes, "COLD enc MEMORY PATTERN ONLY lds-dma 8, nt stores");
    addr(k_pattern_enc<10, 2>, enc_bytes, "COLD enc MEMORY PATTERN ONLY lds-dma 10, nt stores");
    for (uint32_t gp : {1280u, 2560u}) {
      vars.push_back({"COLD enc lds-dma 10 pipelined persistent, nt stores, grid " + std::to_string(gp), enc_bytes, [=]() {
        hipLaunchKernelGGL((k_encode_gp<10, 3, 2, 10>), dim3(gp), dim3(256), 0, 0, rot[(*cnt)++ & 3]); }, {}});
      vars.push_back({"COLD enc lds-dma 6 pipelined persistent, nt stores, grid " + std::to_string(gp), enc_bytes, [=]() {
        hipLaunchKernelGGL((k_encode_gp<10, 3, 2, 6>), dim3(gp), dim3(256), 0, 0, rot[(*cnt)++ & 3]); }, {}});
    }
    pairr(k_encode_g<10, 3, 2, 10>, k_apply_p<10, 1, 3>, "COLD pair enc lds-dma 10 + dec nt3 reg");
    pairr(k_encode_c<10, 3, 3>, k_apply_p<10, 1, 3>, "COLD pair enc nt3 reg + dec nt3 reg");
    pairr(k_encode_c<10, 3, 3>, k_apply_p<10, 1, 3, 1, 1, 4, true, 0, 10>, "COLD pair enc nt3 reg + dec lds-dma");
    pairr(k_encode_g<10, 3, 0, 8>, k_apply_p<10, 1, 1>, "COLD pair old production");
    pairr(k_encode_g<10, 3, 2, 8>, k_apply_p<10, 1, 3, 1, 1, 4, true, 0, 10>, "COLD pair enc lds-dma 8 + dec lds-dma");
    pairr(k_encode_g<10, 3, 2, 8>, k_apply_p<10, 1, 3>, "COLD pair production (enc lds-dma 8 + dec nt3 reg, nt stores both)");
    pairr(k_encode_g<10, 3, 2, 8>, k_apply_p<10, 1, 1>, "COLD pair nt stores encode");
    {  // out-of-place reconstruct pattern: erased rows to a separate [4][G][pitch] batch
      std::vector<Batch> roto(rot);
      for (auto& b : roto) {
        uint8_t* ob;
        CK(hipMalloc(&ob, 4 * G * pitch));
        CK(hipMemset(ob, 0, 4 * G * pitch));
        b.status = reinterpret_cast<int8_t*>(ob);
      }
      const uint32_t grid = (pl.items + 255) / 256;
      std::vector<Batch> rotk(roto);  // the product kernels' own out-of-place form (Batch::out)
      for (auto& b : rotk) {
        b.out = reinterpret_cast<uint8_t*>(b.status);
        b.status = nullptr;
        b.ogstride = pitch;
        b.orstride = G * pitch;
      }
      // round 5 (LDPOL mode): load policy -- plain survivor loads with nt stores
      vars.push_back({"LDPOL dec INTO production k_apply_p nt3 (nt loads + stores)", dec_bytes, [=]() {
        hipLaunchKernelGGL((k_apply_p<10, 1, 3>), dim3(grid), dim3(256), 0, 0, rotk[(*cnt)++ & 3]); }, {}});
      vars.push_back({"LDPOL dec INTO k_apply_p nt2 (plain loads, nt stores)", dec_bytes, [=]() {
        hipLaunchKernelGGL((k_apply_p<10, 1, 2>), dim3(grid), dim3(256), 0, 0, rotk[(*cnt)++ & 3]); }, {}});
      vars.push_back({"LDPOL enc production k_encode_g<10,3,2,8,256,13>", enc_bytes, [=]() {
        hipLaunchKernelGGL((k_encode_g<10, 3, 2, 8, 256, 13>), dim3(grid), dim3(256), 0, 0, rot[(*cnt)++ & 3]); }, {}});
      vars.push_back({"LDPOL pair production (enc + dec INTO nt3)", enc_bytes + dec_bytes, [=]() {
        const int r = (*cnt)++ & 3;
        hipLaunchKernelGGL((k_encode_g<10, 3, 2, 8, 256, 13>), dim3(grid), dim3(256), 0, 0, rot[r]);
        hipLaunchKernelGGL((k_apply_p<10, 1, 3>), dim3(grid), dim3(256), 0, 0, rotk[r]); }, {}});
      vars.push_back({"LDPOL pair enc + dec INTO nt2 (plain survivor loads)", enc_bytes + dec_bytes, [=]() {
        const int r = (*cnt)++ & 3;
        hipLaunchKernelGGL((k_encode_g<10, 3, 2, 8, 256, 13>), dim3(grid), dim3(256), 0, 0, rot[r]);
        hipLaunchKernelGGL((k_apply_p<10, 1, 2>), dim3(grid), dim3(256), 0, 0, rotk[r]); }, {}});
      vars.push_back({"COLD dec INTO production k_apply_p nt3", dec_bytes, [=]() {
        hipLaunchKernelGGL((k_apply_p<10, 1, 3>), dim3(grid), dim3(256), 0, 0, rotk[(*cnt)++ & 3]); }, {}});
      vars.push_back({"COLD dec INTO k_apply_p lds-dma 10", dec_bytes, [=]() {
        hipLaunchKernelGGL((k_apply_p<10, 1, 3, 1, 1, 4, true, 0, 10>), dim3(grid), dim3(256), 0, 0, rotk[(*cnt)++ & 3]); }, {}});
      vars.push_back({"COLD dec INTO k_apply_p lds-dma 8", dec_bytes, [=]() {
        hipLaunchKernelGGL((k_apply_p<10, 1, 3, 1, 1, 4, true, 0, 8>), dim3(grid), dim3(256), 0, 0, rotk[(*cnt)++ & 3]); }, {}});
      vars.push_back({"COLD dec INTO k_apply_p nt1 (plain stores)", dec_bytes, [=]() {
        hipLaunchKernelGGL((k_apply_p<10, 1, 1>), dim3(grid), dim3(256), 0, 0, rotk[(*cnt)++ & 3]); }, {}});
      vars.push_back({"COLD dec INTO k_apply_p emax3", dec_bytes, [=]() {
        hipLaunchKernelGGL((k_apply_p<10, 1, 3, 1, 1, 3>), dim3(grid), dim3(256), 0, 0, rotk[(*cnt)++ & 3]); }, {}});
      vars.push_back({"COLD dec MEMORY PATTERN ONLY nt3, OUT-OF-PLACE outputs", dec_bytes, [=]() {
        hipLaunchKernelGGL((k_pattern_rec<3, false, true>), dim3(grid), dim3(256), 0, 0, roto[(*cnt)++ & 3]); }, {}});
      vars.push_back({"COLD dec MEMORY PATTERN ONLY lds-dma nt stores, OUT-OF-PLACE outputs", dec_bytes, [=]() {
        hipLaunchKernelGGL((k_pattern_rec<3, true, true>), dim3(grid), dim3(256), 0, 0, roto[(*cnt)++ & 3]); }, {}});
    }
    {  // occupancy sweep (round 2): extra dynamic LDS per block caps the blocks per CU, so fewer
       // requests are in flight -- does a lower load on the DRAM banks help the mixed stream pattern?
      const uint32_t grid = (pl.items + 255) / 256;
      std::vector<Batch> rotk(rot);
      for (auto& b : rotk) {
        uint8_t* ob;
        CK(hipMalloc(&ob, 4 * G * pitch));
        b.out = ob;
        b.ogstride = pitch;
        b.orstride = G * pitch;
      }
      for (uint32_t bpc : {5u, 4u, 3u, 2u}) {  // blocks per CU (k_encode_g: 32 KiB static LDS each)
        const uint32_t extra = bpc == 5 ? 0u : (160u * 1024u / bpc - 32u * 1024u - 1024u);  // exactly bpc fit
        vars.push_back({"COLD OCC enc production, " + std::to_string(bpc) + " blocks/CU", enc_bytes, [=]() {
          hipLaunchKernelGGL((k_encode_g<10, 3, 2, 8>), dim3(grid), dim3(256), extra, 0, rot[(*cnt)++ & 3]); }, {}});
      }
      auto occ_extra = [](uint32_t bpc, uint32_t static_kib) {  // dynamic LDS so that bpc blocks fit a CU
        return 160u * 1024u / bpc - static_kib * 1024u - 1024u;  // exactly bpc blocks fit
      };
      vars.push_back({"COLD OCC2 enc lds-dma 10 rows (40 KiB: 4 blocks/CU natively)", enc_bytes, [=]() {
        hipLaunchKernelGGL((k_encode_g<10, 3, 2, 10>), dim3(grid), dim3(256), 0, 0, rot[(*cnt)++ & 3]); }, {}});
      for (uint32_t bpc : {6u, 5u, 4u}) {
        const uint32_t extra = occ_extra(bpc, 24);
        vars.push_back({"COLD OCC2 enc lds-dma 6 rows, " + std::to_string(bpc) + " blocks/CU", enc_bytes, [=]() {
          hipLaunchKernelGGL((k_encode_g<10, 3, 2, 6>), dim3(grid), dim3(256), extra, 0, rot[(*cnt)++ & 3]); }, {}});
      }
      for (uint32_t bpc : {8u, 6u, 5u, 4u, 3u}) {  // all rows to registers (62 VGPRs: 8 waves/SIMD)
        const uint32_t extra = bpc == 8 ? 0u : occ_extra(bpc, 0);
        vars.push_back({"COLD OCC2 enc nt3 registers, " + std::to_string(bpc) + " blocks/CU", enc_bytes, [=]() {
          hipLaunchKernelGGL((k_encode_c<10, 3, 3>), dim3(grid), dim3(256), extra, 0, rot[(*cnt)++ & 3]); }, {}});
      }
      // the bench step: encode then reconstruct_into of the same batch, old vs new encode occupancy
      vars.push_back({"COLD OCC STEP enc 8-row stage (5 blocks/CU) + dec INTO", enc_bytes + dec_bytes, [=]() {
        const int r = (*cnt)++ & 3;
        hipLaunchKernelGGL((k_encode_g<10, 3, 2, 8>), dim3(grid), dim3(256), 0, 0, rot[r]);
        hipLaunchKernelGGL((k_apply_p<10, 1, 3>), dim3(grid), dim3(256), 0, 0, rotk[r]); }, {}});
      vars.push_back({"COLD OCC STEP enc 10-row stage (4 blocks/CU, production) + dec INTO", enc_bytes + dec_bytes, [=]() {
        const int r = (*cnt)++ & 3;
        hipLaunchKernelGGL((k_encode_g<10, 3, 2, 8, 256, 10>), dim3(grid), dim3(256), 0, 0, rot[r]);
        hipLaunchKernelGGL((k_apply_p<10, 1, 3>), dim3(grid), dim3(256), 0, 0, rotk[r]); }, {}});
      vars.push_back({"COLD OCC enc 10-row stage (4 blocks/CU) alone", enc_bytes, [=]() {
        hipLaunchKernelGGL((k_encode_g<10, 3, 2, 8, 256, 10>), dim3(grid), dim3(256), 0, 0, rot[(*cnt)++ & 3]); }, {}});
      vars.push_back({"COLD OCC enc 13-row stage (3 blocks/CU) alone", enc_bytes, [=]() {
        hipLaunchKernelGGL((k_encode_g<10, 3, 2, 8, 256, 13>), dim3(grid), dim3(256), 0, 0, rot[(*cnt)++ & 3]); }, {}});
      vars.push_back({"COLD OCC STEP enc 13-row stage (3 blocks/CU) + dec INTO", enc_bytes + dec_bytes, [=]() {
        const int r = (*cnt)++ & 3;
        hipLaunchKernelGGL((k_encode_g<10, 3, 2, 8, 256, 13>), dim3(grid), dim3(256), 0, 0, rot[r]);
        hipLaunchKernelGGL((k_apply_p<10, 1, 3>), dim3(grid), dim3(256), 0, 0, rotk[r]); }, {}});
      vars.push_back({"COLD OCC3 enc 13-row stage, 10 rows by LDS-DMA", enc_bytes, [=]() {
        hipLaunchKernelGGL((k_encode_g<10, 3, 2, 10, 256, 13>), dim3(grid), dim3(256), 0, 0, rot[(*cnt)++ & 3]); }, {}});
      vars.push_back({"COLD OCC3 enc 13-row stage, 6 rows by LDS-DMA", enc_bytes, [=]() {
        hipLaunchKernelGGL((k_encode_g<10, 3, 2, 6, 256, 13>), dim3(grid), dim3(256), 0, 0, rot[(*cnt)++ & 3]); }, {}});
      vars.push_back({"COLD OCC3 enc 13-row stage, 4 rows by LDS-DMA", enc_bytes, [=]() {
        hipLaunchKernelGGL((k_encode_g<10, 3, 2, 4, 256, 13>), dim3(grid), dim3(256), 0, 0, rot[(*cnt)++ & 3]); }, {}});
      vars.push_back({"COLD OCC3 enc 13-row stage, 8 rows, plain stores", enc_bytes, [=]() {
        hipLaunchKernelGGL((k_encode_g<10, 3, 0, 8, 256, 13>), dim3(grid), dim3(256), 0, 0, rot[(*cnt)++ & 3]); }, {}});
      for (uint32_t bpc : {4u, 3u}) {
        const uint32_t x = 160u * 1024u / bpc - 1024u;
        vars.push_back({"COLD OCC3 enc nt3 registers, exactly " + std::to_string(bpc) + " blocks/CU", enc_bytes, [=]() {
          hipLaunchKernelGGL((k_encode_c<10, 3, 3>), dim3(grid), dim3(256), x, 0, rot[(*cnt)++ & 3]); }, {}});
      }
      {
        const uint32_t g512 = (pl.items + 511) / 512;
        vars.push_back({"COLD OCC3 enc block 512, 8 rows, 13-row stage (1 block = 8 waves/CU... 104 KiB)", enc_bytes, [=]() {
          hipLaunchKernelGGL((k_encode_g<10, 3, 2, 8, 512, 13>), dim3(g512), dim3(512), 0, 0, rot[(*cnt)++ & 3]); }, {}});
        const uint32_t g128 = (pl.items + 127) / 128;
        vars.push_back({"COLD OCC3 enc block 128, 8 rows, 13-row stage (26 KiB: 6 blocks = 12 waves/CU)", enc_bytes, [=]() {
          hipLaunchKernelGGL((k_encode_g<10, 3, 2, 8, 128, 13>), dim3(g128), dim3(128), 0, 0, rot[(*cnt)++ & 3]); }, {}});
      }
      for (uint32_t bpc : {5u, 4u, 3u}) {  // the compute-free encode pattern (8 LDS-DMA rows: 32 KiB)
        const uint32_t x = bpc == 5 ? 0u : (160u * 1024u / bpc - 32u * 1024u - 1024u);
        vars.push_back({"COLD OCC PATTERN enc (no GF), exactly " + std::to_string(bpc) + " blocks/CU", enc_bytes, [=]() {
          hipLaunchKernelGGL((k_pattern_enc<8, 2>), dim3(grid), dim3(256), x, 0, rot[(*cnt)++ & 3]); }, {}});
      }
      {  // 2 KiB per wave per row (2 chunks per lane): fewer distinct DRAM pages in flight per byte
        const uint32_t g2 = (pl.items + 511) / 512;
        for (uint32_t bpc : {4u, 3u, 2u}) {
          const uint32_t x = 160u * 1024u / bpc - 1024u;
          vars.push_back({"COLD OCC4 enc 2 chunks/lane nt3, exactly " + std::to_string(bpc) + " blocks/CU", enc_bytes,
                          [=]() { hipLaunchKernelGGL((k_encode_cpt<2, 3>), dim3(g2), dim3(256), x, 0, rot[(*cnt)++ & 3]); },
                          {}});
        }
        vars.push_back({"COLD OCC4 enc 2 chunks/lane nt3, natural", enc_bytes,
                        [=]() { hipLaunchKernelGGL((k_encode_cpt<2, 3>), dim3(g2), dim3(256), 0, 0, rot[(*cnt)++ & 3]); }, {}});
      }
      vars.push_back({"COLD OCC enc 20-row stage (2 blocks/CU) alone", enc_bytes, [=]() {
        hipLaunchKernelGGL((k_encode_g<10, 3, 2, 8, 256, 20>), dim3(grid), dim3(256), 0, 0, rot[(*cnt)++ & 3]); }, {}});
      for (uint32_t bpc : {4u, 3u}) {  // survivors by LDS-DMA (10 rows: 40 KiB, 4 blocks/CU natively)
        const uint32_t extra = bpc == 4 ? 0u : (160u * 1024u / bpc - 40u * 1024u - 1024u);
        vars.push_back({"COLD OCC dec INTO lds-dma 10, " + std::to_string(bpc) + " blocks/CU", dec_bytes, [=]() {
          hipLaunchKernelGGL((k_apply_p<10, 1, 3, 1, 1, 4, true, 0, 10>), dim3(grid), dim3(256), extra, 0,
                             rotk[(*cnt)++ & 3]); }, {}});
      }
      for (uint32_t bpc : {5u, 4u, 3u}) {  // survivors 0-7 by LDS-DMA (32 KiB)
        const uint32_t extra = bpc == 5 ? 0u : (160u * 1024u / bpc - 32u * 1024u - 1024u);
        vars.push_back({"COLD OCC dec INTO lds-dma 8, " + std::to_string(bpc) + " blocks/CU", dec_bytes, [=]() {
          hipLaunchKernelGGL((k_apply_p<10, 1, 3, 1, 1, 4, true, 0, 8>), dim3(grid), dim3(256), extra, 0,
                             rotk[(*cnt)++ & 3]); }, {}});
      }
      for (uint32_t bpc : {5u, 4u, 3u, 2u}) {  // k_apply_p into: VGPR-limited to 5 blocks/CU
        const uint32_t extra = bpc == 5 ? 0u : (160u * 1024u / bpc - 1024u);  // exactly bpc fit
        vars.push_back({"COLD OCC dec INTO production, " + std::to_string(bpc) + " blocks/CU", dec_bytes, [=]() {
          hipLaunchKernelGGL((k_apply_p<10, 1, 3>), dim3(grid), dim3(256), extra, 0, rotk[(*cnt)++ & 3]); }, {}});
      }
    }
    {  // canonical survivor slots (same kernels, descriptor table with slot r = row r)
      std::vector<Batch> rotc(rot);
      for (auto& b : rotc) b.desc = dtabc;
      const uint32_t grid = (pl.items + 255) / 256;
      vars.push_back({"COLD dec perm nt3 (production kernel), CANON slots", dec_bytes, [=]() {
        hipLaunchKernelGGL((k_apply_p<10, 1, 3>), dim3(grid), dim3(256), 0, 0, rotc[(*cnt)++ & 3]); }, {}});
      vars.push_back({"COLD dec MEMORY PATTERN ONLY nt3, CANON slots", dec_bytes, [=]() {
        hipLaunchKernelGGL((k_pattern_rec<3>), dim3(grid), dim3(256), 0, 0, rotc[(*cnt)++ & 3]); }, {}});
      vars.push_back({"COLD dec perm lds-dma, nt stores, CANON slots", dec_bytes, [=]() {
        hipLaunchKernelGGL((k_apply_p<10, 1, 3, 1, 1, 4, true, 0, 10>), dim3(grid), dim3(256), 0, 0, rotc[(*cnt)++ & 3]); }, {}});
      vars.push_back({"COLD pair production, CANON slots", enc_bytes + dec_bytes, [=]() {
        const Batch& b = rotc[(*cnt)++ & 3];
        hipLaunchKernelGGL((k_encode_g<10, 3, 2, 8>), dim3(grid), dim3(256), 0, 0, b);
        hipLaunchKernelGGL((k_apply_p<10, 1, 3>), dim3(grid), dim3(256), 0, 0, b); }, {}});
      // bit-exact check: canonical-slot table == first-d table, erased rows clobbered before each run
      std::vector<uint8_t> h1(G * n * pitch), h2(G * n * pitch);
      auto clob_run = [&](const Batch& b, std::vector<uint8_t>& out) {
        CK(hipMemcpy(buf, h.data(), h.size(), hipMemcpyHostToDevice));
        hipLaunchKernelGGL((k_encode_c<10, 3, 1>), dim3(grid), dim3(256), 0, 0, pl);
        for (uint64_t g = 0; g < G; g += 97)  // a sample of groups gets garbage in its erased rows
          for (int r = 0; r < n; ++r)
            if (!(hm[g] >> r & 1)) CK(hipMemset(buf + r * pl.rstride + g * pl.gstride, 0xee, S));
        hipLaunchKernelGGL((k_apply_p<10, 1, 3>), dim3(grid), dim3(256), 0, 0, b);
        CK(hipMemcpy(out.data(), buf, out.size(), hipMemcpyDeviceToHost));
      };
      Batch bc = pl; bc.desc = dtabc;
      clob_run(pl, h1);
      clob_run(bc, h2);
      CK(hipMemcpy(buf, h.data(), h.size(), hipMemcpyHostToDevice));
      size_t ndiff = 0;
      for (size_t i = 0; i < h1.size(); ++i) ndiff += h1[i] != h2[i];
      printf("{\"check\":\"k_apply_p CANON slots == first-d slots\",\"equal\":%s,\"diff_bytes\":%zu}\n",
             ndiff ? "false" : "true", ndiff);
      fflush(stdout);
    }
    {  // PROBE (timing only; writes the pitch padding): S = pitch, so every row's
       // tail chunk is a full 16-B store and no 128-B line is partially written
       // by a group's row end.  Same chunks, items and grid as production.
      std::vector<Batch> rotf(rot);
      for (auto& b : rotf) b.S = static_cast<uint32_t>(pitch);
      const uint32_t grid = (pl.items + 255) / 256;
      vars.push_back({"COLD enc production, PROBE full tail chunks (S=pitch)", enc_bytes, [=]() {
        hipLaunchKernelGGL((k_encode_g<10, 3, 2, 8>), dim3(grid), dim3(256), 0, 0, rotf[(*cnt)++ & 3]); }, {}});
      vars.push_back({"COLD dec production, PROBE full tail chunks (S=pitch)", dec_bytes, [=]() {
        hipLaunchKernelGGL((k_apply_p<10, 1, 3>), dim3(grid), dim3(256), 0, 0, rotf[(*cnt)++ & 3]); }, {}});
    }
  }
  if (!cold) {
  // LDS-DMA (global_load_lds_dwordx4 nt) row loads; profiles/r1/kvariants_xcd_rstride.jsonl
  // holds the row-stride sweep (+-2%, kept at G * pitch)
  add(k_encode_g<10, 3, 0>, pl, enc_bytes, "enc planar lds-dma nt");
  add(k_encode_g<10, 3, 0, 8>, pl, enc_bytes, "enc planar lds-dma nt 8 rows + 2 reg");
  add(k_encode_g<10, 3, 2, 8>, pl, enc_bytes, "enc planar lds-dma nt 8 rows + 2 reg, nt stores (production)");
  vars.push_back({"enc planar nt3, 2 chunks per lane", enc_bytes, [=]() {
    hipLaunchKernelGGL((k_encode_cpt<2, 3>), dim3((pl.items + 511) / 512), dim3(256), 0, 0, pl); }, {}});
  add(k_apply_p<10, 1, 3>, pl, dec_bytes, "dec planar perm nt3 (production)");
  add(k_encode_g<10, 3, 0, 9>, pl, enc_bytes, "enc planar lds-dma nt 9 rows + 1 reg");
  add(k_encode_g<10, 3, 0, 7>, pl, enc_bytes, "enc planar lds-dma nt 7 rows + 3 reg");
  {
    const uint32_t g128 = (pl.items + 127) / 128, g512 = (pl.items + 511) / 512;
    vars.push_back({"enc planar lds-dma nt 8 rows, block 128", enc_bytes,
                    [=]() { hipLaunchKernelGGL((k_encode_g<10, 3, 0, 8, 128>), dim3(g128), dim3(128), 0, 0, pl); }, {}});
    vars.push_back({"enc planar lds-dma nt 8 rows, block 512", enc_bytes,
                    [=]() { hipLaunchKernelGGL((k_encode_g<10, 3, 0, 8, 512>), dim3(g512), dim3(512), 0, 0, pl); }, {}});
    vars.push_back({"enc planar lds-dma nt 8 rows, block 64", enc_bytes,
                    [=]() { hipLaunchKernelGGL((k_encode_g<10, 3, 0, 8, 64>), dim3((pl.items + 63) / 64), dim3(64), 0, 0, pl); }, {}});
  }
  add(k_encode_g<10, 3, 0, 6>, pl, enc_bytes, "enc planar lds-dma nt 6 rows + 4 reg");
  add(k_encode_g<10, 3, 0, 5>, pl, enc_bytes, "enc planar lds-dma nt 5 rows + 5 reg");
  add(k_encode_g<10, 3, 0, 3>, pl, enc_bytes, "enc planar lds-dma nt 3 rows + 7 reg");
  add(k_apply_p<10, 1, 1, 1, 1, 4, true, 0, 10>, pl, dec_bytes, "dec planar perm lds-dma asm-collect");
  add(k_apply_p<10, 1, 1, 1, 1, 4, true, 0, 8>, pl, dec_bytes, "dec planar perm lds-dma asm-collect 8 rows + 2 reg");
  pair(k_encode_g<10, 3, 0, 8>, k_apply_p<10, 1, 1, 1, 1, 4, true, 0, 8>, pl, "pair planar lds-dma enc 8 + perm lds-dma 8");
  pair(k_encode_g<10, 3, 0, 8>, k_apply_p<10, 1, 1, 1, 1, 4, true, 0, 10>, pl, "pair planar lds-dma enc 8 + perm lds-dma 10");
  add(k_pattern_rec<1, true>, pl, dec_bytes, "dec planar MEMORY PATTERN ONLY lds-dma nt (xor, no GF)");
  pair(k_encode_g<10, 3, 0, 8>, k_apply_p<10, 1, 1>, pl, "pair planar lds-dma enc 8 rows + perm-nt1");

  }  // !cold

  {  // LDS-DMA variants must reproduce the register-load kernels bit for bit
    const uint32_t grid = (pl.items + 255) / 256;
    std::vector<uint8_t> hc(h), h1(h.size()), h2(h.size());
    for (uint64_t g = 0; g < G; ++g)
      for (int r = 0; r < n; ++r)
        if (!(hm[g] >> r & 1)) memset(hc.data() + r * pl.rstride + g * pl.gstride, 0xee, S);
    auto run_cmp = [&](const char* nm, auto ka, auto kb) {
      CK(hipMemcpy(buf, hc.data(), hc.size(), hipMemcpyHostToDevice));
      hipLaunchKernelGGL(ka, dim3(grid), dim3(256), 0, 0, pl);
      CK(hipMemcpy(h1.data(), buf, h1.size(), hipMemcpyDeviceToHost));
      CK(hipMemcpy(buf, hc.data(), hc.size(), hipMemcpyHostToDevice));
      hipLaunchKernelGGL(kb, dim3(grid), dim3(256), 0, 0, pl);
      CK(hipMemcpy(h2.data(), buf, h2.size(), hipMemcpyDeviceToHost));
      printf("{\"check\":\"%s\",\"equal\":%s,\"changed\":%s}\n", nm, h1 == h2 ? "true" : "false",
             h1 == hc ? "false" : "true");
      fflush(stdout);
    };
    run_cmp("k_encode_g == k_encode_c", k_encode_c<10, 3, 1>, k_encode_g<10, 3, 0>);
    run_cmp("k_encode_g<8> == k_encode_c", k_encode_c<10, 3, 1>, k_encode_g<10, 3, 0, 8>);


    {
      CK(hipMemcpy(buf, hc.data(), hc.size(), hipMemcpyHostToDevice));
      hipLaunchKernelGGL((k_encode_c<10, 3, 1>), dim3(grid), dim3(256), 0, 0, pl);
      CK(hipMemcpy(h1.data(), buf, h1.size(), hipMemcpyDeviceToHost));
      CK(hipMemcpy(buf, hc.data(), hc.size(), hipMemcpyHostToDevice));
      hipLaunchKernelGGL((k_encode_cpt<2, 3>), dim3((pl.items + 511) / 512), dim3(256), 0, 0, pl);
      CK(hipMemcpy(h2.data(), buf, h2.size(), hipMemcpyDeviceToHost));
      printf("{\"check\":\"k_encode_cpt<2> == k_encode_c\",\"equal\":%s}\n", h1 == h2 ? "true" : "false");
    }
    run_cmp("k_apply_p lds-dma asm-collect == k_apply_p", k_apply_p<10, 1, 1>, k_apply_p<10, 1, 1, 1, 1, 4, true, 0, 10>);
    run_cmp("k_apply_p lds-dma 8 == k_apply_p", k_apply_p<10, 1, 1>, k_apply_p<10, 1, 1, 1, 1, 4, true, 0, 8>);
    CK(hipMemcpy(buf, h.data(), h.size(), hipMemcpyHostToDevice));
  }

  {  // k_apply_p must reproduce k_apply_w bit for bit (random masks, planar)
    const uint32_t grid = (pl.items + 255) / 256;
    Batch b1 = pl;
    b1.pass = (pl.items + 63u) / 64u * 64u;
    std::vector<uint8_t> h1(h.size()), h2(h.size());
    hipLaunchKernelGGL((k_apply_w<10, 1, 3, 1>), dim3(grid), dim3(256), 0, 0, b1);
    CK(hipMemcpy(h1.data(), buf, h.size(), hipMemcpyDeviceToHost));
    CK(hipMemset(buf, 0x5a, h.size() / 2));
    CK(hipMemcpy(buf, h1.data(), h.size(), hipMemcpyHostToDevice));
    // clobber erased rows so the check sees fresh outputs
    for (uint64_t g = 0; g < G; ++g)
      for (int r = 0; r < n; ++r)
        if (!(hm[g] >> r & 1)) CK(hipMemset(buf + r * pl.rstride + g * pl.gstride, 0xee, S));
    hipLaunchKernelGGL((k_apply_p<10, 1, 3, 1>), dim3(grid), dim3(256), 0, 0, pl);
    CK(hipMemcpy(h2.data(), buf, h.size(), hipMemcpyDeviceToHost));
    printf("{\"check\":\"k_apply_p<1> == k_apply_w\",\"equal\":%s}\n", h1 == h2 ? "true" : "false");
    for (uint64_t g = 0; g < G; ++g)
      for (int r = 0; r < n; ++r)
        if (!(hm[g] >> r & 1)) CK(hipMemset(buf + r * pl.rstride + g * pl.gstride, 0xee, S));
    hipLaunchKernelGGL((k_apply_p<10, 1, 3, 2>), dim3(grid), dim3(256), 0, 0, pl);
    CK(hipMemcpy(h2.data(), buf, h.size(), hipMemcpyDeviceToHost));
    printf("{\"check\":\"k_apply_p<2> == k_apply_w\",\"equal\":%s}\n", h1 == h2 ? "true" : "false");
    fflush(stdout);
  }
  if (const char* f = getenv("KVAR_FILTER")) {  // '|'-separated substrings; keep matching variants
    std::vector<Var> kept;
    std::string fs(f);
    for (auto& v : vars) {
      size_t a = 0;
      while (a <= fs.size()) {
        const size_t b = std::min(fs.find('|', a), fs.size());
        if (b > a && v.name.find(fs.substr(a, b - a)) != std::string::npos) { kept.push_back(v); break; }
        a = b + 1;
      }
    }
    vars.swap(kept);
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vars) { v.go(); }
  CK(hipDeviceSynchronize());
  // Cold mode: before every sample, an untimed plain-load sweep of 768 MB
  // evicts the Infinity Cache, so no variant pays for the dirty lines the
  // previous one left (the write-back happens inside the sweep).
  uint8_t* flushbuf = nullptr;
  const uint64_t flush_n16 = (768ull << 20) / 16;
  if (cold) {
    CK(hipMalloc(&flushbuf, flush_n16 * 16 + 64));
    CK(hipMemset(flushbuf, 1, flush_n16 * 16));
  }
  for (int r = 0; r < rounds; ++r)
    for (auto& v : vars) {
      if (cold) hipLaunchKernelGGL(k_flush_read, dim3((flush_n16 + 255) / 256), dim3(256), 0, 0,
                                   reinterpret_cast<const u32x4*>(flushbuf), reinterpret_cast<uint32_t*>(flushbuf), flush_n16);
      CK(hipEventRecord(e0));
      for (int i = 0; i < 5; ++i) v.go();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.t.push_back(ms / 5);
    }
  for (auto& v : vars) {
    std::sort(v.t.begin(), v.t.end());
    float med = v.t[v.t.size() / 2], mn = v.t[0];
    printf("{\"variant\":\"%s\",\"median_us\":%.2f,\"min_us\":%.2f,\"GBps\":%.1f}\n", v.name.c_str(), med * 1e3,
           mn * 1e3, v.bytes / (med * 1e-3) / 1e9);
  }
  return 0;
}
