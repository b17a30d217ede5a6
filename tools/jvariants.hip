// A/B timing of jumbo (32+8)x9000 kernel variants, planar layout, 8192 groups.
// Not product code: includes the kernel TU.  One JSON line per variant.
#include "../ugo_amd/csrc/fec_kernels.hip"
#include "fec_experiments.hpp"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

using namespace ugo;
using namespace ugo::kern;

// k_apply_qa (wave-aligned groups) is production since round 2 (fec_kernels.hip).

// ---------------------------------------------- k_apply_gq (A/B only)
// Round-2 attempt at fusing k_prepare into the jumbo apply (DESIGN_HISTORY.md §3.4):
// bit-exact, but 634.6 us against 569.3 us for k_prepare + k_apply_q
// (jvar_r2h.jsonl).  Kept here, out of the product, as the record.
constexpr uint32_t kMaxDescBytes = 1024;
// Group-per-block reconstruct for d + p > 16 (MODE 2) with the descriptor
// build fused in: block b owns group g0 + b.  The block stages M and the GF
// tables in LDS, wave 0 builds the group's descriptor there (prep_wave), and
// after one barrier the block streams the group's chunks exactly as
// k_apply_q does -- every descriptor word read from LDS and made scalar by
// readfirstlane, the coefficient tables read as scalar loads.  One launch
// instead of k_prepare + k_apply_q, no workspace, and no wave ever spans two
// groups (no per-lane table pick).  A block of W waves covers the group's C
// chunks in P = ceil(C / 256) passes (W = ceil(C / 64P): 3 waves x 3 passes
// for the 563 chunks of a 9000-B row, 97.7% of the lanes busy).  Survivor
// rows are read with buffer loads: a wave-uniform resource per row (SALU
// address arithmetic) and the lane's chunk offset.
__device__ __forceinline__ uint32_t lds_u32(const uint32_t* p) {  // LDS word -> SGPR (uniform address)
  return __builtin_amdgcn_readfirstlane(*p);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const uint8_t* base, uint64_t off) {
  const uint64_t a64 = reinterpret_cast<uint64_t>(base) + off;
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a64));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(a64 >> 32));
  void* p = reinterpret_cast<void*>((static_cast<uint64_t>(hi) << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(p, 0, 0x7fffffff, 0x00020000);
}

template <int NT>
__device__ __forceinline__ V4 bload16(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, (NT & 1) ? 2 : 0));
  return V4{{v.x, v.y, v.z, v.w}};
}


// PREP (A/B only, tools/jvariants.hip): 1 = copy a descriptor k_prepare left
// in pr.desc instead of building it (isolates the cost of the build).
template <int EMAX, int NT, int RING = 4, int PREP = 0>
__global__ __launch_bounds__(256) void k_apply_gq(Batch a, Prep pr) {
  static_assert(RING == 4, "one coefficient word per input quad");
  __shared__ PrepShared sh;
  __shared__ PrepWave s;
  __shared__ uint32_t sdesc[kMaxDescBytes / 4];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t g = a.g0 + blockIdx.x;
  const uint32_t d = a.d;
  if constexpr (PREP == 0) {
    prep_stage(pr, sh, threadIdx.x, blockDim.x);
    __syncthreads();
    if (wave == 0) prep_wave(pr, g, reinterpret_cast<uint8_t*>(sdesc), sh, s, lane);
  } else {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(pr.desc + (g - pr.g_desc0) * pr.desc_stride);
    for (uint32_t i = threadIdx.x; i < pr.desc_stride / 4; i += blockDim.x) sdesc[i] = src[i];
  }
  __syncthreads();
  const uint32_t hdr = lds_u32(&sdesc[0]);
  const uint32_t st = (hdr >> 16) & 0xffu;
  const uint32_t e = st ? 0u : (a.data_only ? ((hdr >> 8) & 0xffu) : (hdr & 0xffu));
  const bool wst = a.status != nullptr && threadIdx.x == 0;
  if (e == 0) {  // block-uniform
    if (wst) a.status[g] = static_cast<int8_t>(st);
    return;
  }
  // survivors: the first d present rows in index order (the rows prep_wave
  // lists), popped from the mask with scalar bit scans
  const uint64_t m64 = pr.present[g] & pr.nmask;
  const uint32_t mlo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(m64));  // (int -> u32: no sign
  const uint32_t mhi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(m64 >> 32));  //  extension)
  const uint64_t mask = static_cast<uint64_t>(mhi) << 32 | mlo;
  const uint8_t* gbase = a.base + g * a.gstride;
  // The tables are read through the constant address space: this kernel
  // stores to LDS (the descriptor) and to global memory (status, outputs)
  // before it reads them, which would make plain global reads per-lane vector
  // loads; constant reads are scalar loads whatever was stored before (the
  // tables are never written by any kernel).
  const ctab_t ctab = (ctab_t)a.mult;
  const uint32_t cbase = 4 + a.dpad + a.epad;  // byte offset of coefficient row 0 (multiple of 4)
  const uint8_t* orow = reinterpret_cast<const uint8_t*>(sdesc) + 4 + a.dpad;
  for (uint32_t c0 = 0; c0 < a.chunks; c0 += blockDim.x) {  // passes (block-uniform)
    const uint32_t c = c0 + threadIdx.x;
    const bool live = c < a.chunks;
    const uint32_t voff = live ? c * 16u : 0u;  // idle lanes load chunk 0 and store nothing
    uint64_t rem = mask;                         // present rows not yet loaded
    auto load_next = [&](uint32_t k) -> V4 {
      if (k >= d) return V4{{0u, 0u, 0u, 0u}};  // uniform: every lane takes the same rows
      const uint32_t r = static_cast<uint32_t>(__builtin_ctzll(rem));
      rem &= rem - 1;
      return bload16<NT>(row_rsrc(gbase, static_cast<uint64_t>(r) * a.rstride), voff);
    };
    V4 ring[RING];
#pragma unroll
    for (int j = 0; j < RING; ++j) ring[j] = load_next(j);
    V4 acc[EMAX];
#pragma unroll
    for (int i = 0; i < EMAX; ++i) acc[i] = V4{{0u, 0u, 0u, 0u}};
    for (uint32_t k0 = 0; k0 < d; k0 += RING) {
#pragma unroll
      for (int j = 0; j < RING; j += 2) {
        const uint32_t k = k0 + j;
        uint32_t s0[4], s1[4], s2[4], r0[4], r1[4], r2[4];
        p_sel(ring[j], s0, s1, s2);
        p_sel(ring[j + 1], r0, r1, r2);
        ring[j] = load_next(k + RING);
        ring[j + 1] = load_next(k + RING + 1);
#pragma unroll
        for (int i = 0; i < EMAX; ++i) {
          if (i >= static_cast<int>(e)) continue;
          const uint32_t cw = lds_u32(&sdesc[(cbase + i * a.dpad + k0) >> 2]);  // inputs k0..k0+3
          const ctab_t tA = ctab + 8u * ((cw >> (8 * j)) & 0xffu);
          const ctab_t tB = ctab + 8u * ((cw >> (8 * (j + 1))) & 0xffu);
          uint32_t t[5], u[5];
#pragma unroll
          for (int q = 0; q < 5; ++q) {
            t[q] = tA[q];
            u[q] = tB[q];
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            uint32_t y = xor3(acc[i].v[q], perm(t[1], t[0], s0[q]), perm(t[3], t[2], s1[q]));
            y = xor3(y, perm(0u, t[4], s2[q]), perm(u[1], u[0], r0[q]));
            acc[i].v[q] = xor3(y, perm(u[3], u[2], r1[q]), perm(0u, u[4], r2[q]));
          }
        }
      }
    }
    if (live) {
      uint8_t* gp = a.base + g * a.gstride + voff;
      const uint32_t nb = a.S - voff;
#pragma unroll
      for (int i = 0; i < EMAX; ++i) {
        if (i >= static_cast<int>(e)) continue;
        const uint32_t r = (lds_u32(reinterpret_cast<const uint32_t*>(orow) + (i >> 2)) >> (8 * (i & 3))) & 0xffu;
        store16<NT>(out_row(a, gp, g, voff, r, i), acc[i], nb);
      }
    }
  }
  if (wst) a.status[g] = 0;
}



// Floor of k_prepare (A/B only): the same grid, staging and mask read, and a
// header store per group, no descriptor build.
__global__ __launch_bounds__(64 * kPrepWaves) void k_prep_floor(Prep a, uint32_t groups) {
  __shared__ PrepShared sh;
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
  prep_stage(a, sh, threadIdx.x, 64 * kPrepWaves);
  __syncthreads();
  const uint32_t gl = blockIdx.x * kPrepWaves + w;
  if (gl >= groups) return;
  const uint64_t g = a.g0 + gl;
  const uint64_t mask = a.present[g] & a.nmask;
  if (lane == 0)
    *reinterpret_cast<uint32_t*>(a.desc + (g - a.g_desc0) * a.desc_stride) = __popcll(mask) | sh.M[lane] << 24;
}

int main(int argc, char** argv) {
  const int d = 32, p = 8, n = 40;
  const uint32_t S = 9000, pitch = 9008;
  const uint64_t G = argc > 1 ? atoll(argv[1]) : 8192;
  const int rounds = argc > 2 ? atoi(argv[2]) : 9;
  const uint32_t dpad = 32, epad = 8, stride = ((4 + dpad + epad + p * dpad + 15) / 16 * 16);
  uint8_t* buf;
  CK(hipMalloc(&buf, G * n * pitch));
  std::vector<uint8_t> h(G * n * pitch);
  uint64_t st = 0x5EED;
  for (auto& b : h) { st = st * 6364136223846793005ull + 1442695040888963407ull; b = st >> 56; }
  CK(hipMemcpy(buf, h.data(), h.size(), hipMemcpyHostToDevice));
  // matrix, encode descriptor, perm tables, gf tables
  std::vector<uint8_t> M(n * d), scratch(n * d + 3 * d * d);
  gf::build_matrix(d, p, M.data(), scratch.data());
  std::vector<uint8_t> ed(stride + 64, 0);
  ed[0] = p;
  for (int i = 0; i < d; ++i) ed[4 + i] = i;
  for (int i = 0; i < p; ++i) ed[4 + dpad + i] = d + i;
  for (int i = 0; i < p; ++i)
    for (int k = 0; k < d; ++k) ed[4 + dpad + epad + i * dpad + k] = M[(d + i) * d + k];
  std::vector<uint8_t> gfv(1024 + 8192, 0);
  memcpy(gfv.data(), gf::kTables.exp, 512);
  memcpy(gfv.data() + 512, gf::kTables.log, 256);
  gf::perm_tables(gfv.data() + 1024);
  uint8_t *d_ed, *d_gf, *d_M, *d_work;
  uint64_t* masks;
  CK(hipMalloc(&d_ed, ed.size()));
  CK(hipMalloc(&d_gf, gfv.size()));
  CK(hipMalloc(&d_M, M.size()));
  CK(hipMalloc(&d_work, G * stride + 64));
  CK(hipMalloc(&masks, G * 8));
  CK(hipMemcpy(d_ed, ed.data(), ed.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_gf, gfv.data(), gfv.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_M, M.data(), M.size(), hipMemcpyHostToDevice));
  // mixed erasures e ~ U[0,8], positions uniform among the 40 shards
  std::vector<uint64_t> hm(G);
  double dec_rows = 0;
  for (uint64_t g = 0; g < G; ++g) {
    st = st * 6364136223846793005ull + 1442695040888963407ull;
    int e = (st >> 33) % 9;
    uint64_t m = (1ull << n) - 1;
    while (__builtin_popcountll(((1ull << n) - 1) & ~m) < e) {
      st = st * 6364136223846793005ull + 1442695040888963407ull;
      m &= ~(1ull << ((st >> 33) % n));
    }
    hm[g] = m;
    if (e > 0) dec_rows += d + e;  // a group with no erasure moves nothing
  }
  CK(hipMemcpy(masks, hm.data(), G * 8, hipMemcpyHostToDevice));
  Batch a{};
  a.base = buf; a.gstride = pitch; a.rstride = G * pitch; a.nmask = (1ull << n) - 1; a.S = S;
  a.chunks = (S + 15) / 16; a.items = G * a.chunks; a.desc_stride = stride; a.d = d;
  a.dpad = dpad; a.epad = epad; a.mult = reinterpret_cast<const uint32_t*>(d_gf + 1024);
  Batch ae = a;  // MODE 0: encode through the descriptor kernels
  ae.desc = d_ed;
  Batch ar = a;  // MODE 2: per-group descriptors
  ar.desc = d_work; ar.present = masks; ar.g_desc0 = 0;
  Prep pr{};
  pr.desc = d_work; pr.present = masks; pr.M = d_M; pr.gf_exp = d_gf; pr.gf_log = d_gf + 512; pr.g0 = 0;
  pr.g_desc0 = 0; pr.nmask = a.nmask; pr.desc_stride = stride; pr.d = d; pr.n = n; pr.dpad = dpad; pr.epad = epad;
  CK(hipMemset(d_work, 0xEE, G * stride));
  CK(launch_prepare(pr, G, 0));
  CK(hipDeviceSynchronize());
  const double enc_bytes = double(G) * n * S, dec_bytes = dec_rows * S;
  const uint32_t grid = (a.items + 255) / 256;
  struct Var { std::string name; double bytes; std::function<void()> go; std::vector<float> t; };
  std::vector<Var> vars;
  auto add = [&](auto kern, const Batch& b, double bytes, std::string nm) {
    vars.push_back({nm, bytes, [=]() { hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, b); }, {}});
  };
  add(k_encode_c<32, 8, 1>, a, enc_bytes, "enc const-network nt1");
  add(k_encode_c<32, 8, 3>, a, enc_bytes, "enc const-network nt3");
  add(k_encode_g<32, 8, 2, 8>, a, enc_bytes, "enc const-network lds-dma 8 rows, nt stores (production since round 2)");
  add(k_encode_g<32, 8, 2, 16>, a, enc_bytes, "enc const-network lds-dma 16 rows, nt stores (round-1 production)");
  add(k_encode_g<32, 8, 0, 8>, a, enc_bytes, "enc const-network lds-dma 8 rows");
  const size_t kFr = vars.size();
  add(k_encode_fr<32, 8, 2, 8>, a, enc_bytes, "enc FOUR-RUSSIANS network (blocks of 3), lds-dma 8 rows, nt stores");
  add(k_encode_fr<32, 8, 2, 8, 256, 8, 3>, a, enc_bytes, "enc FOUR-RUSSIANS network (blocks of 3), lds-dma 8 rows, nt stores, 3 waves/SIMD");
  add(k_encode_fr<32, 8, 2, 8, 256, 8, 2>, a, enc_bytes, "enc FOUR-RUSSIANS network (blocks of 3), lds-dma 8 rows, nt stores, 2 waves/SIMD");
  add(k_encode_frs<32, 8, 2, 8, 256, 8, 1>, a, enc_bytes, "enc FOUR-RUSSIANS SEQ dwords, lds-dma 8 rows, nt stores");
  add(k_encode_frs<32, 8, 2, 8, 256, 8, 3>, a, enc_bytes, "enc FOUR-RUSSIANS SEQ dwords, lds-dma 8 rows, nt stores, 3 waves/SIMD");
  add(k_encode_frs<32, 8, 2, 16, 256, 16, 3>, a, enc_bytes, "enc FOUR-RUSSIANS SEQ dwords, lds-dma 16 rows, nt stores, 3 waves/SIMD");
  add(k_encode_frs<32, 8, 2, 12, 256, 12, 3>, a, enc_bytes, "enc FOUR-RUSSIANS SEQ dwords, lds-dma 12 rows, nt stores, 3 waves/SIMD");
  add(k_encode_frs<32, 8, 2, 16, 256, 16, 3, 4>, a, enc_bytes, "enc FOUR-RUSSIANS SEQ dwords, BLOCKS OF 4, lds-dma 16 rows, nt stores");
  add(k_encode_frs<32, 8, 2, 16, 256, 16, 3, 2>, a, enc_bytes, "enc FOUR-RUSSIANS SEQ dwords, BLOCKS OF 2, lds-dma 16 rows, nt stores");
  add(k_encode_frs<32, 8, 2, 20, 256, 20, 3>, a, enc_bytes, "enc FOUR-RUSSIANS SEQ dwords, lds-dma 20 rows, nt stores, 3 waves/SIMD");
  {
    const uint32_t g128 = (a.items + 127) / 128, g64 = (a.items + 63) / 64;
    vars.push_back({"enc FOUR-RUSSIANS SEQ dwords, lds-dma 16 rows, 128-thread blocks", enc_bytes, [=]() {
      hipLaunchKernelGGL((k_encode_frs<32, 8, 2, 16, 128, 16, 3>), dim3(g128), dim3(128), 0, 0, a); }, {}});
    vars.push_back({"enc FOUR-RUSSIANS SEQ dwords, lds-dma 20 rows, 128-thread blocks", enc_bytes, [=]() {
      hipLaunchKernelGGL((k_encode_frs<32, 8, 2, 20, 128, 20, 3>), dim3(g128), dim3(128), 0, 0, a); }, {}});
    vars.push_back({"enc FOUR-RUSSIANS SEQ dwords, lds-dma 24 rows, 64-thread blocks", enc_bytes, [=]() {
      hipLaunchKernelGGL((k_encode_frs<32, 8, 2, 24, 64, 24, 3>), dim3(g64), dim3(64), 0, 0, a); }, {}});
    vars.push_back({"enc FOUR-RUSSIANS SEQ dwords, lds-dma 32 rows, 64-thread blocks", enc_bytes, [=]() {
      hipLaunchKernelGGL((k_encode_frs<32, 8, 2, 32, 64, 32, 3>), dim3(g64), dim3(64), 0, 0, a); }, {}});
  }
  add(k_apply_q<8, 0, 1, 1, 4>, ae, enc_bytes, "enc perm-tables streaming ring4 nt1");
  add(k_apply_q<8, 0, 1, 1, 8>, ae, enc_bytes, "enc perm-tables streaming ring8 nt1");
  add(k_apply_q<8, 0, 3, 1, 4>, ae, enc_bytes, "enc perm-tables streaming ring4 nt3 (generic-code encode, production)");
  add(k_apply_q<8, 0, 3, 1, 2>, ae, enc_bytes, "enc perm-tables streaming ring2 nt3");
  add(k_apply_q<8, 2, 1, 1, 4>, ar, dec_bytes, "dec perm streaming ring4 nt1");
  add(k_apply_q<8, 2, 1, 1, 8>, ar, dec_bytes, "dec perm streaming ring8 nt1");
  add(k_apply_q<8, 2, 3, 1, 4>, ar, dec_bytes, "dec perm streaming ring4 nt3 (production)");
  add(k_apply_q<8, 2, 3, 1, 2>, ar, dec_bytes, "dec perm streaming ring2 nt3");
  {  // residency caps (round 2): dynamic LDS so that exactly `bpc` blocks fit a CU
    auto cap = [](uint32_t bpc, uint32_t static_kib) { return 160u * 1024u / bpc - static_kib * 1024u - 1024u; };
    for (uint32_t bpc : {4u, 3u, 2u}) {
      const uint32_t x = cap(bpc, 0);
      vars.push_back({"dec perm streaming (production), OCC " + std::to_string(bpc) + " blocks/CU", dec_bytes, [=]() {
        hipLaunchKernelGGL((k_apply_q<8, 2, 3, 1, 4>), dim3(grid), dim3(256), x, 0, ar); }, {}});
    }
    for (uint32_t bpc : {4u, 3u, 2u, 1u}) {
      const uint32_t x = cap(bpc, 32);
      vars.push_back({"enc const-network lds-dma 8 rows, nt stores, OCC " + std::to_string(bpc) + " blocks/CU", enc_bytes,
                      [=]() { hipLaunchKernelGGL((k_encode_g<32, 8, 2, 8>), dim3(grid), dim3(256), x, 0, a); }, {}});
    }
    {
      const uint32_t x = cap(1, 64);
      vars.push_back({"enc const-network lds-dma 16 rows, nt stores, OCC 1 block/CU", enc_bytes,
                      [=]() { hipLaunchKernelGGL((k_encode_g<32, 8, 2, 16>), dim3(grid), dim3(256), x, 0, a); }, {}});
    }
  }
  {  // wave-aligned groups: item = g * 576 + chunk
    Batch aa = ar;
    aa.items = G * ((a.chunks + 63) / 64 * 64);
    const uint32_t ga = (aa.items + 255) / 256;
    vars.push_back({"dec perm streaming ring4 nt3, WAVE-ALIGNED groups (k_apply_qa)", dec_bytes, [=]() {
      hipLaunchKernelGGL((k_apply_qa<8, 2, 3, 4>), dim3(ga), dim3(256), 0, 0, aa); }, {}});
    vars.push_back({"dec k_apply_qa ring4 waves_per_eu 5", dec_bytes, [=]() {
      hipLaunchKernelGGL((k_apply_qa<8, 2, 3, 4, 5>), dim3(ga), dim3(256), 0, 0, aa); }, {}});
    vars.push_back({"dec k_apply_qa ring2 (production since round 2)", dec_bytes, [=]() {
      hipLaunchKernelGGL((k_apply_qa<8, 2, 3, 2>), dim3(ga), dim3(256), 0, 0, aa); }, {}});
    vars.push_back({"dec k_apply_qa ring2 waves_per_eu 5", dec_bytes, [=]() {
      hipLaunchKernelGGL((k_apply_qa<8, 2, 3, 2, 5>), dim3(ga), dim3(256), 0, 0, aa); }, {}});
    vars.push_back({"dec k_apply_qa ring2 waves_per_eu 6", dec_bytes, [=]() {
      hipLaunchKernelGGL((k_apply_qa<8, 2, 3, 2, 6>), dim3(ga), dim3(256), 0, 0, aa); }, {}});
    vars.push_back({"dec k_apply_qa ring2 waves_per_eu 7", dec_bytes, [=]() {
      hipLaunchKernelGGL((k_apply_qa<8, 2, 3, 2, 7>), dim3(ga), dim3(256), 0, 0, aa); }, {}});
  }
  add(k_apply_q<8, 2, 0, 1, 4>, ar, dec_bytes, "dec perm streaming ring4 nt0");
  add(k_apply<32, 2, 3>, ar, dec_bytes, "dec masked-horner k_apply nt3 (before)");
  // (round 2: the log-domain build, 21.0 us, against the table-product build with
  // serial loops, 23.8 us, byte-identical descriptors: profiles/r2/jvariants_prepare_v2.jsonl)
  vars.push_back({"k_prepare (8192 groups, production: small tier)", 0.0, [=]() { launch_prepare(pr, G, 0); }, {}});
  vars.push_back({"k_prepare generic tier (EDM 32, 22.9 KiB LDS) on the jumbo code", 0.0, [=]() {
    hipLaunchKernelGGL((k_prepare<32, 64 * 64>), dim3((G + kPrepWaves - 1) / kPrepWaves), dim3(64 * kPrepWaves), 0, 0,
                       pr, static_cast<uint32_t>(G)); }, {}});
  Prep pf = pr;  // own workspace: the timed decode variants read d_work
  CK(hipMalloc(&pf.desc, G * stride + 64));
  vars.push_back({"k_prepare FLOOR (staging + mask read + header store, no build)", 0.0, [=]() {
    hipLaunchKernelGGL(k_prep_floor, dim3((G + kPrepWaves - 1) / kPrepWaves), dim3(64 * kPrepWaves), 0, 0, pf,
                       static_cast<uint32_t>(G)); }, {}});
  {  // fused descriptor build, one group per block (k_apply_gq, A/B only)
    const uint32_t passes = (a.chunks + 255) / 256, bs = 64 * ((a.chunks + 64 * passes - 1) / (64 * passes));
    Batch af = a;
    af.present = masks;
    vars.push_back({"dec fused k_apply_gq (production)", dec_bytes, [=]() {
      hipLaunchKernelGGL((k_apply_gq<8, 3>), dim3(G), dim3(bs), 0, 0, af, pr); }, {}});
    vars.push_back({"dec fused k_apply_gq, PROBE descriptor copied from k_prepare's workspace", dec_bytes, [=]() {
      hipLaunchKernelGGL((k_apply_gq<8, 3, 4, 1>), dim3(G), dim3(bs), 0, 0, af, pr); }, {}});
    vars.push_back({"dec k_prepare + k_apply_q (round-2 production before k_apply_qa)", dec_bytes, [=]() {
      launch_prepare(pr, G, 0);
      hipLaunchKernelGGL((k_apply_q<8, 2, 3, 1, 4>), dim3(grid), dim3(256), 0, 0, ar); }, {}});
    {
      Batch aa = ar;
      aa.items = G * ((a.chunks + 63) / 64 * 64);
      const uint32_t ga = (aa.items + 255) / 256;
      vars.push_back({"dec k_prepare + k_apply_qa ring2 (production)", dec_bytes, [=]() {
        launch_prepare(pr, G, 0);
        hipLaunchKernelGGL((k_apply_qa<8, 2, 3, 2>), dim3(ga), dim3(256), 0, 0, aa); }, {}});
      // two halves: the second half's descriptor build runs on a side stream
      // while the first half is applied
      hipStream_t s2;
      hipEvent_t ev0, evB;
      CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
      CK(hipEventCreateWithFlags(&ev0, hipEventDisableTiming));
      CK(hipEventCreateWithFlags(&evB, hipEventDisableTiming));
      const uint64_t H = G / 2;
      Prep pA = pr, pB = pr;
      pB.g0 = H;
      Batch aA = ar, aB = ar;
      aA.items = H * ((a.chunks + 63) / 64 * 64);
      aB.g0 = H;
      aB.items = (G - H) * ((a.chunks + 63) / 64 * 64);
      const uint32_t gA = (aA.items + 255) / 256, gB = (aB.items + 255) / 256;
      vars.push_back({"dec OVERLAP: prepare(half 2) on a side stream during apply(half 1)", dec_bytes, [=]() {
        (void)hipEventRecord(ev0, 0);
        (void)hipStreamWaitEvent(s2, ev0, 0);
        (void)launch_prepare(pB, static_cast<uint32_t>(G - H), s2);
        (void)hipEventRecord(evB, s2);
        (void)launch_prepare(pA, static_cast<uint32_t>(H), 0);
        hipLaunchKernelGGL((k_apply_qa<8, 2, 3, 2>), dim3(gA), dim3(256), 0, 0, aA);
        (void)hipStreamWaitEvent(0, evB, 0);
        hipLaunchKernelGGL((k_apply_qa<8, 2, 3, 2>), dim3(gB), dim3(256), 0, 0, aB); }, {}});
      vars.push_back({"dec two halves, one stream (prepare A, apply A, prepare B, apply B)", dec_bytes, [=]() {
        (void)launch_prepare(pA, static_cast<uint32_t>(H), 0);
        hipLaunchKernelGGL((k_apply_qa<8, 2, 3, 2>), dim3(gA), dim3(256), 0, 0, aA);
        (void)launch_prepare(pB, static_cast<uint32_t>(G - H), 0);
        hipLaunchKernelGGL((k_apply_qa<8, 2, 3, 2>), dim3(gB), dim3(256), 0, 0, aB); }, {}});
    }
  }
  // encode variants must agree: run const then perm encode over the same data
  auto same_rows = [&](const std::vector<uint8_t>& x, const std::vector<uint8_t>& y) {  // bytes [0, S) only
    for (uint64_t r = 0; r < uint64_t(n); ++r)
      for (uint64_t g = 0; g < G; ++g)
        if (memcmp(&x[r * a.rstride + g * pitch], &y[r * a.rstride + g * pitch], S)) return false;
    return true;
  };
  {
    std::vector<uint8_t> h1(h.size()), h2(h.size());
    vars[0].go();
    CK(hipMemcpy(h1.data(), buf, h.size(), hipMemcpyDeviceToHost));
    CK(hipMemset(buf + size_t(d) * a.rstride, 0, size_t(p) * a.rstride));
    vars[2].go();
    CK(hipMemcpy(h2.data(), buf, h.size(), hipMemcpyDeviceToHost));
    printf("{\"check\":\"perm encode == const encode\",\"equal\":%s}\n", same_rows(h1, h2) ? "true" : "false");
    for (size_t f = kFr; f < kFr + 14; ++f) {
      CK(hipMemset(buf + size_t(d) * a.rstride, 0, size_t(p) * a.rstride));
      vars[f].go();
      CK(hipMemcpy(h2.data(), buf, h.size(), hipMemcpyDeviceToHost));
      printf("{\"check\":\"%s == const encode\",\"equal\":%s}\n", vars[f].name.c_str(),
             same_rows(h1, h2) ? "true" : "false");
    }
    std::vector<uint8_t> h3(h.size());
    vars[4].go();  // reconstruct of a consistent batch rewrites erased rows with the same bytes
    CK(hipMemcpy(h3.data(), buf, h.size(), hipMemcpyDeviceToHost));
    printf("{\"check\":\"reconstruct of codewords is idempotent\",\"equal\":%s}\n", same_rows(h3, h1) ? "true" : "false");
    // every decode variant recovers garbage-filled erased rows to the codewords
    std::vector<uint8_t> hc = h1;
    for (uint64_t g = 0; g < G; ++g)
      for (int r = 0; r < n; ++r)
        if (!((hm[g] >> r) & 1)) memset(&hc[r * a.rstride + g * pitch], 0xA5, S);
    for (auto& v : vars) {
      if (v.name.rfind("dec", 0) != 0) continue;
      CK(hipMemcpy(buf, hc.data(), hc.size(), hipMemcpyHostToDevice));
      v.go();
      CK(hipMemcpy(h3.data(), buf, h.size(), hipMemcpyDeviceToHost));
      printf("{\"check\":\"%s recovers erased rows\",\"equal\":%s}\n", v.name.c_str(), same_rows(h3, h1) ? "true" : "false");
    }
    fflush(stdout);
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vars) v.go();
  CK(hipDeviceSynchronize());
  for (int r = 0; r < rounds; ++r)
    for (auto& v : vars) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < 3; ++i) v.go();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.t.push_back(ms / 3);
    }
  for (auto& v : vars) {
    std::sort(v.t.begin(), v.t.end());
    const float med = v.t[v.t.size() / 2];
    printf("{\"variant\":\"%s\",\"median_us\":%.2f,\"min_us\":%.2f,\"GBps\":%.1f}\n", v.name.c_str(), med * 1e3,
           v.t[0] * 1e3, v.bytes / (med * 1e-3) / 1e9);
  }
  return 0;
}
