// qaprobe.hip -- jumbo reconstruct A/B (round 3): production k_apply_qa
// against k_apply_qb with each of its three overhead cuts on / off, on the
// (32+8)x9000 batch of BASELINE configs[4] (8,192 groups, planar, e ~ U[0,8]
// mixed erasures, per-group descriptors from k_prepare).  Every variant first
// recovers garbage-filled erased rows of an encoded batch, checked on the
// device against the encoded batch; then interleaved rounds, median per
// variant (cdna_hip_programming.md §5.4 rule 24).
// Usage: qaprobe [groups] [rounds] [row_pad] [nbuf] [planar|gm] [contig]: row_pad bytes added to the
// planar row stride (G * pitch + row_pad), to see whether the row streams'
// relative alignment (G * 9008 = 2^17 * 563 at 8,192 groups) matters.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/qaprobe tools/qaprobe.hip
// Round-3 results: profiles/r3/qaprobe_r3m.jsonl (DESIGN_HISTORY.md §3.4 "Jumbo floor").
// Not product code: it includes the kernel TU to instantiate the variants.
#include "../ugo_amd/csrc/fec_kernels.hip"
#include "fec_experiments.hpp"

#include <algorithm>
#include <cstdio>
#include <functional>
#include <string>
#include <vector>

using namespace ugo;
using namespace ugo::kern;

#include "ab_common.hpp"

__global__ void k_fill(uint8_t* p, uint64_t n16, uint64_t seed) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += gridDim.x * 256ull) {
    uint64_t s = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
    s ^= s >> 31; s *= 0xBF58476D1CE4E5B9ull; s ^= s >> 27;
    uint64_t t = s * 0x94D049BB133111EBull; t ^= t >> 29;
    reinterpret_cast<uint64_t*>(p)[2 * i] = s;
    reinterpret_cast<uint64_t*>(p)[2 * i + 1] = t;
  }
}

// erased rows of every group overwritten with 0xA5
__global__ void k_garble(uint8_t* base, const uint64_t* masks, uint64_t G, uint32_t n, uint64_t rstride,
                         uint64_t gstride, uint32_t S) {
  const uint64_t g = blockIdx.x;
  if (g >= G) return;
  for (uint32_t r = 0; r < n; ++r)
    if (!((masks[g] >> r) & 1))
      for (uint32_t b = threadIdx.x; b < S; b += blockDim.x) base[r * rstride + g * gstride + b] = 0xA5;
}

// rows [r0, r1) of every group overwritten with 0xA5 over their S bytes
__global__ void k_garble_rows(uint8_t* base, uint32_t r0, uint32_t r1, uint64_t G, uint64_t rstride, uint64_t gstride,
                              uint32_t S) {
  const uint64_t g = blockIdx.x;
  if (g >= G) return;
  for (uint32_t r = r0; r < r1; ++r)
    for (uint32_t b = threadIdx.x; b < S; b += blockDim.x) base[r * rstride + g * gstride + b] = 0xA5;
}

__global__ void k_cmp(const uint8_t* x, const uint8_t* y, uint64_t n16, unsigned long long* bad) {
  unsigned long long nb = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += gridDim.x * 256ull) {
    const uint4 a = reinterpret_cast<const uint4*>(x)[i], b = reinterpret_cast<const uint4*>(y)[i];
    nb += (a.x != b.x) + (a.y != b.y) + (a.z != b.z) + (a.w != b.w);
  }
  if (nb) atomicAdd(bad, nb);
}

int main(int argc, char** argv) {
  const int d = 32, p = 8, n = 40;
  const uint32_t S = 9000, pitch = 9008;
  const uint64_t G = argc > 1 ? atoll(argv[1]) : 8192;
  const int rounds = argc > 2 ? atoi(argv[2]) : 11;
  const uint32_t dpad = 32, epad = 8, stride = ((4 + dpad + epad + p * dpad + 15) / 16 * 16);
  const uint64_t row_pad = argc > 3 ? atoll(argv[3]) : 0;
  // layout: planar [row][G][pitch] (default) or group-major [G][row][pitch] ("gm")
  const bool gm = argc > 5 && std::string(argv[5]) == "gm";
  const uint64_t rstride = gm ? pitch : G * pitch + row_pad;
  const uint64_t gstride = gm ? uint64_t(n) * pitch : pitch;
  const uint64_t bytes = gm ? G * n * pitch : n * rstride;
  uint8_t *buf, *ref, *d_gf, *d_M, *d_work, *d_ed;
  uint64_t* masks;
  unsigned long long* bad;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&ref, bytes));
  CK(hipMalloc(&bad, 8));
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, buf, bytes / 16, 99ull);
  std::vector<uint8_t> M(n * d), scratch(n * d + 3 * d * d);
  gf::build_matrix(d, p, M.data(), scratch.data());
  std::vector<uint8_t> gfv(1024 + 8192, 0);
  memcpy(gfv.data(), gf::kTables.exp, 512);
  memcpy(gfv.data() + 512, gf::kTables.log, 256);
  gf::perm_tables(gfv.data() + 1024);
  CK(hipMalloc(&d_gf, gfv.size()));
  CK(hipMalloc(&d_M, M.size()));
  CK(hipMalloc(&d_work, G * stride + 64));
  CK(hipMalloc(&d_ed, stride + 64));
  CK(hipMalloc(&masks, G * 8));
  CK(hipMemcpy(d_gf, gfv.data(), gfv.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_M, M.data(), M.size(), hipMemcpyHostToDevice));
  std::vector<uint64_t> hm(G);
  double dec_rows = 0;
  uint64_t st = 0x5EED;
  for (uint64_t g = 0; g < G; ++g) {
    st = st * 6364136223846793005ull + 1442695040888963407ull;
    int e = (st >> 33) % 9;
    uint64_t m = (1ull << n) - 1;
    while (__builtin_popcountll(((1ull << n) - 1) & ~m) < e) {
      st = st * 6364136223846793005ull + 1442695040888963407ull;
      m &= ~(1ull << ((st >> 33) % n));
    }
    hm[g] = m;
    if (e > 0) dec_rows += d + e;
  }
  CK(hipMemcpy(masks, hm.data(), G * 8, hipMemcpyHostToDevice));
  Batch a{};
  a.base = buf; a.gstride = gstride; a.rstride = rstride; a.nmask = (1ull << n) - 1; a.S = S;
  a.chunks = (S + 15) / 16; a.items = G * a.chunks; a.desc_stride = stride; a.d = d;
  a.dpad = dpad; a.epad = epad; a.mult = reinterpret_cast<const uint32_t*>(d_gf + 1024);
  CK(launch_encode_const(d, p, a, 0));  // codewords
  CK(hipMemcpy(ref, buf, bytes, hipMemcpyDeviceToDevice));
  Prep pr{};
  pr.desc = d_work; pr.present = masks; pr.M = d_M; pr.gf_exp = d_gf; pr.gf_log = d_gf + 512; pr.g0 = 0;
  pr.g_desc0 = 0; pr.nmask = a.nmask; pr.desc_stride = stride; pr.d = d; pr.n = n; pr.dpad = dpad; pr.epad = epad;
  CK(launch_prepare(pr, G, 0));
  Batch aa = a;
  aa.desc = d_work; aa.present = masks; aa.g_desc0 = 0;
  aa.items = G * ((a.chunks + 63) / 64 * 64);
  const uint32_t ga = (aa.items + 255) / 256;
  const uint32_t ga8 = (ga + 7) / 8 * 8;  // OPT & 32 grids: a multiple of 8
  CK(hipDeviceSynchronize());
  const double dec_bytes = dec_rows * S;
  struct Var { std::string name; std::function<void()> go; std::vector<float> t; };
  std::vector<Var> vars;
  vars.push_back({"k_apply_qa ring2 (round 2)", [=]() {
    hipLaunchKernelGGL((k_apply_qa<8, 2, 3, 2>), dim3(ga), dim3(256), 0, 0, aa); }, {}});
  vars.push_back({"k_apply_qb OPT 1 (uniform desc)", [=]() { hipLaunchKernelGGL((k_apply_qb<8, 2, 3, 1>), dim3(ga), dim3(256), 0, 0, aa); }, {}});
  vars.push_back({"k_apply_qb OPT 3 (+ saddr loads; 72 VGPRs, 7 waves/SIMD)", [=]() { hipLaunchKernelGGL((k_apply_qb<8, 2, 3, 3>), dim3(ga), dim3(256), 0, 0, aa); }, {}});
  vars.push_back({"k_apply_qb OPT 7 (+ unrolled ring; 96 VGPRs, 5 waves/SIMD)", [=]() { hipLaunchKernelGGL((k_apply_qb<8, 2, 3, 7>), dim3(ga), dim3(256), 0, 0, aa); }, {}});
  vars.push_back({"k_apply_ql LDS-DMA ring 8", [=]() { hipLaunchKernelGGL((k_apply_ql<8, 2, 8>), dim3(ga), dim3(256), 0, 0, aa); }, {}});
  vars.push_back({"k_apply_ql LDS-DMA ring 8, one pair per iteration", [=]() { hipLaunchKernelGGL((k_apply_ql<8, 2, 8, false>), dim3(ga), dim3(256), 0, 0, aa); }, {}});
  vars.push_back({"k_apply_ql LDS-DMA ring 4", [=]() { hipLaunchKernelGGL((k_apply_ql<8, 2, 4>), dim3(ga), dim3(256), 0, 0, aa); }, {}});
  vars.push_back({"MEMORY PATTERN ONLY of k_apply_qb OPT 7 (inputs XORed, no products; wrong bytes)", [=]() {
    hipLaunchKernelGGL((k_apply_qb<8, 2, 3, 15>), dim3(ga), dim3(256), 0, 0, aa); }, {}});
  vars.push_back({"k_apply_qb OPT 39 (7 + XCD-contiguous blocks)", [=]() {
    hipLaunchKernelGGL((k_apply_qb<8, 2, 3, 39>), dim3(ga8), dim3(256), 0, 0, aa); }, {}});
  {
    const uint32_t ge = (a.items + 255) / 256, ge8 = (ge + 7) / 8 * 8;
    vars.push_back({"ENCODE k_encode_frs (production)", [=]() {
      hipLaunchKernelGGL((k_encode_frs<32, 8, kEncJumboNT & 2, kEncJumboLdsRows, 256, kEncJumboLdsRows, 3, kEncJumboFrBlock>),
                         dim3(ge), dim3(256), 0, 0, a); }, {}});
    vars.push_back({"ENCODE k_encode_frs XCD-contiguous blocks", [=]() {
      hipLaunchKernelGGL((k_encode_frs<32, 8, kEncJumboNT & 2, kEncJumboLdsRows, 256, kEncJumboLdsRows, 3, kEncJumboFrBlock, true>),
                         dim3(ge8), dim3(256), 0, 0, a); }, {}});
  }
  vars.push_back({"k_prepare + k_apply_qa (round 2)", [=]() {
    (void)launch_prepare(pr, G, 0);
    hipLaunchKernelGGL((k_apply_qa<8, 2, 3, 2>), dim3(ga), dim3(256), 0, 0, aa); }, {}});
  vars.push_back({"k_prepare + k_apply_qb OPT 3", [=]() {
    (void)launch_prepare(pr, G, 0);
    hipLaunchKernelGGL((k_apply_qb<8, 2, 3, 3>), dim3(ga), dim3(256), 0, 0, aa); }, {}});
  vars.push_back({"k_prepare + k_apply_qb OPT 39 (production)", [=]() {
    (void)launch_prepare(pr, G, 0);
    hipLaunchKernelGGL((k_apply_qb<8, 2, 3, 39>), dim3(ga8), dim3(256), 0, 0, aa); }, {}});
  vars.push_back({"k_prepare + k_apply_qb OPT 7", [=]() {
    (void)launch_prepare(pr, G, 0);
    hipLaunchKernelGGL((k_apply_qb<8, 2, 3, 7>), dim3(ga), dim3(256), 0, 0, aa); }, {}});
  for (auto& v : vars) {  // correctness: garbage in the erased rows, recovered to the codewords
    CK(hipMemcpy(buf, ref, bytes, hipMemcpyDeviceToDevice));
    const bool enc = v.name.rfind("ENCODE", 0) == 0;
    if (enc)  // encode: garbage in every parity row, rebuilt from the data rows
      hipLaunchKernelGGL(k_garble_rows, dim3(static_cast<uint32_t>(G)), dim3(256), 0, 0, buf, uint32_t(d), uint32_t(n), G,
                         a.rstride, a.gstride, S);
    else
      hipLaunchKernelGGL(k_garble, dim3(static_cast<uint32_t>(G)), dim3(256), 0, 0, buf, masks, G, n, a.rstride, a.gstride, S);
    v.go();
    CK(hipMemset(bad, 0, 8));
    hipLaunchKernelGGL(k_cmp, dim3(4096), dim3(256), 0, 0, buf, ref, bytes / 16, bad);
    unsigned long long nbad = 0;
    CK(hipMemcpy(&nbad, bad, 8, hipMemcpyDeviceToHost));
    printf("{\"check\": \"%s recovers garbage-filled erased (encode: parity) rows\", \"mismatched_dwords\": %llu}\n", v.name.c_str(), nbad);
  }
  CK(hipMemcpy(buf, ref, bytes, hipMemcpyDeviceToDevice));
  fflush(stdout);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w)
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
  // placement: the same batch copied into nbuf more allocations of the same
  // size; the memory-pattern-only variant and OPT 7 timed on each
  // (nbuf < 0: |nbuf| copies carved from ONE allocation, 2 MiB apart)
  const int nbuf_arg = argc > 4 ? atoi(argv[4]) : 0;
  const int nbuf = nbuf_arg < 0 ? -nbuf_arg : nbuf_arg;
  // argv[6] == "contig": the copies from hipExtMallocWithFlags(hipDeviceMallocContiguous)
  const bool contig = argc > 6 && std::string(argv[6]) == "contig";
  const uint64_t slot = (bytes + (2u << 20) - 1) / (2u << 20) * (2u << 20);
  uint8_t* arena = nullptr;
  if (nbuf_arg < 0) CK(hipMalloc(&arena, slot * nbuf));
  for (int b = 0; b < nbuf; ++b) {
    uint8_t* cp;
    if (arena) cp = arena + slot * b;
    else if (contig ? hipExtMallocWithFlags(reinterpret_cast<void**>(&cp), bytes, hipDeviceMallocContiguous) != hipSuccess
                    : hipMalloc(&cp, bytes) != hipSuccess) {
      printf("{\"buffer\": %d, \"alloc\": \"failed\"}\n", b + 1);
      break;
    }
    CK(hipMemcpy(cp, buf, bytes, hipMemcpyDeviceToDevice));
    Batch ab = aa;
    ab.base = cp;
    hipPointerAttribute_t at{};
    (void)hipPointerGetAttributes(&at, cp);
    for (int opt : {15, 47, 7, 39}) {
      std::vector<float> t;
      for (int r = 0; r < rounds + 3; ++r) {
        CK(hipEventRecord(e0));
        for (int i = 0; i < 3; ++i) {
          if (opt == 15) hipLaunchKernelGGL((k_apply_qb<8, 2, 3, 15>), dim3(ga), dim3(256), 0, 0, ab);
          else if (opt == 47) hipLaunchKernelGGL((k_apply_qb<8, 2, 3, 47>), dim3(ga8), dim3(256), 0, 0, ab);
          else if (opt == 39) hipLaunchKernelGGL((k_apply_qb<8, 2, 3, 39>), dim3(ga8), dim3(256), 0, 0, ab);
          else hipLaunchKernelGGL((k_apply_qb<8, 2, 3, 7>), dim3(ga), dim3(256), 0, 0, ab);
        }
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 3) t.push_back(ms / 3);
      }
      std::sort(t.begin(), t.end());
      printf("{\"layout\": \"%s\", \"contig\": %d, \"row_pad\": %llu, \"buffer\": %d, \"va\": \"%p\", \"variant\": \"%s\", \"median_us\": %.2f, \"min_us\": %.2f}\n",
             gm ? "group-major" : "planar", contig ? 1 : 0, (unsigned long long)row_pad, b + 1, (void*)cp, opt == 15 ? "MEMORY PATTERN ONLY" : opt == 47 ? "MEMORY PATTERN ONLY, XCD-contiguous blocks"
             : opt == 39 ? "k_apply_qb OPT 39 (7 + XCD-contiguous blocks)" : "k_apply_qb OPT 7",
             t[t.size() / 2] * 1e3, t[0] * 1e3);
    }
    fflush(stdout);
  }
  for (auto& v : vars) {
    std::sort(v.t.begin(), v.t.end());
    const float med = v.t[v.t.size() / 2];
    printf("{\"layout\": \"%s\", \"row_pad\": %llu, \"variant\": \"%s\", \"median_us\": %.2f, \"min_us\": %.2f, \"TBps\": %.3f}\n", gm ? "group-major" : "planar", (unsigned long long)row_pad, v.name.c_str(), med * 1e3,
           v.t[0] * 1e3, dec_bytes / (med * 1e-3) / 1e12);
  }
  return 0;
}
