// bucket_probe.hip -- A/B of a pattern-bucketed schedule for the headline
// reconstruct_into (k_apply_p<10,1,3> writing the erased rows to a separate
// [4][G][pitch] batch), cold regime (4 rotating batches, an untimed 768-MB
// sweep before every sample), interleaved rounds, medians.
//
// Question: uniformly random 2-erasure patterns cost
// ~9% against one fixed pattern, because every row stream mixes reads, skips
// and (in place) writes.  If groups were processed in pattern order -- a
// pre-pass histograms the 78 presence patterns, prefix-sums them and scatters
// a group permutation -- every wave would load the same 10 rows and take the
// pick-free table path, at the price of reading each group's rows as
// scattered 1360-B pieces instead of one sequential stream per row.
//
// Variants (same descriptor table, same outputs):
//   prod random        production kernel, random patterns, identity order
//   prod fixed         production kernel, one pattern for every group (the ideal)
//   perm identity      the permuted kernel with perm[i] = i (indirection cost)
//   perm host-stable   groups sorted by pattern (stable: ascending within a bucket)
//   perm device        permutation from the device counting sort below (unstable)
//   prepass            the device counting sort alone: LDS histogram, scan, scatter
// Check: every permuted run's output batch equals the production output.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/bucket_probe tools/bucket_probe.hip
#include "../ugo_amd/csrc/fec_kernels.hip"

#include <algorithm>
#include <functional>
#include <memory>
#include <numeric>
#include <string>

using namespace ugo;
using namespace ugo::kern;

#include "ab_common.hpp"

// k_apply_p<10, 1 (MODE 1), 3 (nt), 1 (TSEL), 1, 4, PAIR> with position i of the
// launch mapped to group perm[i]: a wave's two positions pA, pB become groups
// gA = perm[pA], gB = perm[pB] (scalar loads), each lane's group is its
// position's.  Outputs go to a.out (reconstruct_into).
template <bool PERM>
__global__ __launch_bounds__(256) void k_apply_perm(Batch a, const uint32_t* __restrict__ perm) {
  constexpr int DMAX = 10, EMAX = 4;
  const uint32_t wfirst = blockIdx.x * 256u + (__builtin_amdgcn_readfirstlane(threadIdx.x) & ~63u);
  const uint32_t item = blockIdx.x * 256u + threadIdx.x;
  if (wfirst >= a.items) return;
  const uint32_t wlast = min(wfirst + 63u, a.items - 1u);
  const uint32_t pA = wfirst / a.chunks, pB = wlast / a.chunks;
  const uint64_t gA = PERM ? perm[pA] : pA, gB = PERM ? perm[pB] : pB;
  const uint8_t* dA = desc_for<1>(a, gA);
  const uint8_t* dB = desc_for<1>(a, gB);
  constexpr int NW = (DMAX + 3) / 4;
  const uint32_t hA = ld32(dA), hB = ld32(dB);
  uint32_t rA[NW], rB[NW];
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    rA[w] = ld32(dA + 4 + 4 * w);
    rB[w] = ld32(dB + 4 + 4 * w);
  }
  const uint32_t oA = ld32(dA + 4 + a.dpad), oB = ld32(dB + 4 + a.dpad);
  const uint32_t eA = ((hA >> 16) & 0xffu) ? 0u : (hA & 0xffu);
  const uint32_t eB = ((hB >> 16) & 0xffu) ? 0u : (hB & 0xffu);
  const uint32_t emax = max(eA, eB);
  if (item >= a.items) return;
  const uint32_t pl = item / a.chunks;
  const bool inB = pl != pA;
  const uint32_t c = item - pl * a.chunks;
  const uint64_t g = inB ? gB : gA;
  const uint32_t e = inB ? eB : eA;
  if (e == 0) return;
  uint32_t mB;
  asm("v_mov_b32 %0, %1" : "=v"(mB) : "v"(inB ? ~0u : 0u));
  uint8_t* gp = a.base + g * a.gstride + static_cast<uint64_t>(c) * 16u;
  const uint32_t nb = a.S - c * 16u;
  V4 x[DMAX];
#pragma unroll
  for (int k = 0; k < DMAX; ++k) {
    const uint32_t rw = inB ? rB[k >> 2] : rA[k >> 2];
    const uint32_t r = (rw >> (8 * (k & 3))) & 0xffu;
    x[k] = load16<3>(gp + static_cast<uint64_t>(r) * a.rstride);
  }
  V4 acc[EMAX];
  if (dA == dB)
    p_accum<DMAX, 0, EMAX, true>(acc, x, a, dA, dA, 0u, emax);
  else
    p_accum<DMAX, 1, EMAX, true>(acc, x, a, dA, dB, mB, emax);
  const uint32_t orows = inB ? oB : oA;
#pragma unroll
  for (int i = 0; i < EMAX; ++i) {
    if (i >= static_cast<int>(e)) continue;
    const uint32_t r = (orows >> (8 * i)) & 0xffu;
    store16<3>(out_row(a, gp, g, c * 16u, r, i), acc[i], nb);
  }
}

// Device counting sort of the groups by presence mask (8192 bins for n = 13).
__global__ __launch_bounds__(256) void k_hist(const uint64_t* __restrict__ masks, uint64_t G, uint64_t nmask,
                                              uint32_t* __restrict__ bins) {
  __shared__ uint32_t h[8192];
  for (uint32_t i = threadIdx.x; i < 8192; i += 256) h[i] = 0;
  __syncthreads();
  for (uint64_t g = blockIdx.x * 256ull + threadIdx.x; g < G; g += gridDim.x * 256ull)
    atomicAdd(&h[masks[g] & nmask], 1u);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < 8192; i += 256)
    if (h[i]) atomicAdd(&bins[i], h[i]);
}

__global__ __launch_bounds__(1024) void k_scan(uint32_t* __restrict__ bins) {  // in place, exclusive, 8192 bins
  __shared__ uint32_t part[1024];
  uint32_t v[8], s = 0;
  for (int j = 0; j < 8; ++j) {
    v[j] = bins[threadIdx.x * 8 + j];
    s += v[j];
  }
  part[threadIdx.x] = s;
  __syncthreads();
  for (uint32_t off = 1; off < 1024; off <<= 1) {
    const uint32_t t = threadIdx.x >= off ? part[threadIdx.x - off] : 0u;
    __syncthreads();
    part[threadIdx.x] += t;
    __syncthreads();
  }
  uint32_t run = part[threadIdx.x] - s;
  for (int j = 0; j < 8; ++j) {
    bins[threadIdx.x * 8 + j] = run;
    run += v[j];
  }
}

__global__ __launch_bounds__(256) void k_scatter(const uint64_t* __restrict__ masks, uint64_t G, uint64_t nmask,
                                                 uint32_t* __restrict__ bins, uint32_t* __restrict__ perm) {
  const uint64_t g = blockIdx.x * 256ull + threadIdx.x;
  if (g < G) perm[atomicAdd(&bins[masks[g] & nmask], 1u)] = static_cast<uint32_t>(g);
}

__global__ __launch_bounds__(256) void k_flush_sweep(const u32x4* __restrict__ a, uint32_t* out, uint64_t n16) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += gridDim.x * 256ull) acc ^= a[i].x;
  if (acc == 0x9e3779b9u) out[0] = acc;
}

int main(int argc, char** argv) {
  const int d = 10, p = 3, n = 13;
  const uint32_t S = 1350, pitch = 1360;
  const uint64_t G = argc > 1 ? atoll(argv[1]) : 65536;
  const int rounds = argc > 2 ? atoi(argv[2]) : 15;
  const uint32_t dpad = 12, epad = 4, stride = 64;
  std::vector<uint8_t> tab;
  build_table(d, p, dpad, epad, stride, tab);
  uint8_t* dtab;
  CK(hipMalloc(&dtab, tab.size()));
  CK(hipMemcpy(dtab, tab.data(), tab.size(), hipMemcpyHostToDevice));
  std::vector<uint8_t> hmul(256 * 32);
  gf::perm_tables(hmul.data());
  uint32_t* dmul;
  CK(hipMalloc(&dmul, hmul.size()));
  CK(hipMemcpy(dmul, hmul.data(), hmul.size(), hipMemcpyHostToDevice));

  // random 2-erasure masks (the bench's C3 workload) and one fixed pattern
  uint64_t st = 0x5EED;
  std::vector<uint64_t> hm(G), hf(G, ((1ull << n) - 1) & ~(1ull << 3) & ~(1ull << 11));
  for (uint64_t g = 0; g < G; ++g) {
    st = st * 6364136223846793005ull + 1442695040888963407ull;
    const int x = (st >> 33) % n, y = (x + 1 + (st >> 40) % (n - 1)) % n;
    hm[g] = ((1ull << n) - 1) & ~(1ull << x) & ~(1ull << y);
  }
  std::vector<uint32_t> hs(G), hid(G);
  std::iota(hid.begin(), hid.end(), 0u);
  hs = hid;
  std::stable_sort(hs.begin(), hs.end(), [&](uint32_t a, uint32_t b) { return hm[a] < hm[b]; });
  uint64_t *dm, *dfix;
  uint32_t *dperm_s, *dperm_id, *dperm_dev, *dbins;
  CK(hipMalloc(&dm, G * 8));
  CK(hipMalloc(&dfix, G * 8));
  CK(hipMalloc(&dperm_s, G * 4));
  CK(hipMalloc(&dperm_id, G * 4));
  CK(hipMalloc(&dperm_dev, G * 4));
  CK(hipMalloc(&dbins, 8192 * 4));
  CK(hipMemcpy(dm, hm.data(), G * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dfix, hf.data(), G * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dperm_s, hs.data(), G * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dperm_id, hid.data(), G * 4, hipMemcpyHostToDevice));
  const uint64_t nmask = (1ull << n) - 1;
  const uint32_t gblocks = static_cast<uint32_t>((G + 255) / 256);
  auto prepass = [=]() {
    (void)hipMemsetAsync(dbins, 0, 8192 * 4, 0);
    hipLaunchKernelGGL(k_hist, dim3(std::min<uint32_t>(gblocks, 256)), dim3(256), 0, 0, dm, G, nmask, dbins);
    hipLaunchKernelGGL(k_scan, dim3(1), dim3(1024), 0, 0, dbins);
    hipLaunchKernelGGL(k_scatter, dim3(gblocks), dim3(256), 0, 0, dm, G, nmask, dbins, dperm_dev);
  };
  prepass();
  CK(hipDeviceSynchronize());
  {  // the device permutation is a permutation sorted by mask
    std::vector<uint32_t> hp(G);
    CK(hipMemcpy(hp.data(), dperm_dev, G * 4, hipMemcpyDeviceToHost));
    std::vector<uint32_t> chk(hp);
    std::sort(chk.begin(), chk.end());
    bool ok = chk == hid;
    for (uint64_t i = 1; i < G && ok; ++i) ok = hm[hp[i - 1]] <= hm[hp[i]];
    printf("{\"check\":\"device counting sort is a mask-sorted permutation\",\"ok\":%s}\n", ok ? "true" : "false");
  }

  // 4 rotating input batches (planar [13][G][pitch]) + their output batches [4][G][pitch]
  const uint64_t bbytes = G * n * pitch, obytes = 4 * G * pitch;
  std::vector<uint8_t> h(bbytes);
  for (auto& b : h) { st = st * 6364136223846793005ull + 1442695040888963407ull; b = st >> 56; }
  Batch base{};
  base.mult = dmul;
  base.gstride = pitch;
  base.rstride = G * pitch;
  base.nmask = nmask;
  base.S = S;
  base.chunks = 85;
  base.items = static_cast<uint32_t>(G * 85);
  base.desc = dtab;
  base.desc_stride = stride;
  base.d = d;
  base.dpad = dpad;
  base.epad = epad;
  base.ogstride = pitch;
  base.orstride = G * pitch;
  std::vector<Batch> rot(4, base);
  for (auto& b : rot) {
    CK(hipMalloc(&b.base, bbytes));
    CK(hipMemcpy(b.base, h.data(), bbytes, hipMemcpyHostToDevice));
    CK(hipMalloc(&b.out, obytes));
    CK(hipMemset(b.out, 0, obytes));
    b.present = dm;
  }
  const uint32_t grid = (base.items + 255) / 256;
  const double bytes = double(G) * 12 * S;
  struct Var { std::string name; double bytes; std::function<void()> go; std::vector<float> t; };
  std::vector<Var> vars;
  auto cnt = std::make_shared<int>(0);
  vars.push_back({"prod random", bytes, [=]() {
    hipLaunchKernelGGL((k_apply_p<10, 1, 3>), dim3(grid), dim3(256), 0, 0, rot[(*cnt)++ & 3]); }, {}});
  vars.push_back({"prod fixed (ideal: one pattern)", bytes, [=]() {
    Batch b = rot[(*cnt)++ & 3];
    b.present = dfix;
    hipLaunchKernelGGL((k_apply_p<10, 1, 3>), dim3(grid), dim3(256), 0, 0, b); }, {}});
  vars.push_back({"perm identity", bytes, [=]() {
    hipLaunchKernelGGL((k_apply_perm<true>), dim3(grid), dim3(256), 0, 0, rot[(*cnt)++ & 3], (const uint32_t*)dperm_id); }, {}});
  vars.push_back({"perm host-stable (bucketed)", bytes, [=]() {
    hipLaunchKernelGGL((k_apply_perm<true>), dim3(grid), dim3(256), 0, 0, rot[(*cnt)++ & 3], (const uint32_t*)dperm_s); }, {}});
  vars.push_back({"perm device (bucketed, unstable)", bytes, [=]() {
    hipLaunchKernelGGL((k_apply_perm<true>), dim3(grid), dim3(256), 0, 0, rot[(*cnt)++ & 3], (const uint32_t*)dperm_dev); }, {}});
  vars.push_back({"perm device + prepass", bytes, [=]() {
    prepass();
    hipLaunchKernelGGL((k_apply_perm<true>), dim3(grid), dim3(256), 0, 0, rot[(*cnt)++ & 3], (const uint32_t*)dperm_dev); }, {}});
  vars.push_back({"prepass alone", 0.0, [=]() { prepass(); (*cnt)++; }, {}});

  {  // bit-exactness: every permuted form writes the production output batch
    std::vector<uint8_t> ref(obytes), got(obytes);
    auto run = [&](std::function<void(const Batch&)> f, std::vector<uint8_t>& out) {
      CK(hipMemset(rot[0].out, 0xee, obytes));
      f(rot[0]);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(out.data(), rot[0].out, obytes, hipMemcpyDeviceToHost));
    };
    run([=](const Batch& b) { hipLaunchKernelGGL((k_apply_p<10, 1, 3>), dim3(grid), dim3(256), 0, 0, b); }, ref);
    for (auto pr : {std::make_pair("identity", dperm_id), std::make_pair("host-stable", dperm_s),
                    std::make_pair("device", dperm_dev)}) {
      run([=](const Batch& b) {
        hipLaunchKernelGGL((k_apply_perm<true>), dim3(grid), dim3(256), 0, 0, b, (const uint32_t*)pr.second); }, got);
      printf("{\"check\":\"perm %s == production\",\"equal\":%s}\n", pr.first, got == ref ? "true" : "false");
    }
    fflush(stdout);
  }

  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vars) v.go();
  CK(hipDeviceSynchronize());
  uint8_t* flushbuf = nullptr;
  const uint64_t flush_n16 = (768ull << 20) / 16;
  CK(hipMalloc(&flushbuf, flush_n16 * 16 + 64));
  CK(hipMemset(flushbuf, 1, flush_n16 * 16));
  for (int r = 0; r < rounds; ++r)
    for (auto& v : vars) {
      hipLaunchKernelGGL(k_flush_sweep, dim3(2048), dim3(256), 0, 0, reinterpret_cast<const u32x4*>(flushbuf),
                         reinterpret_cast<uint32_t*>(flushbuf), flush_n16);
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
    const float med = v.t[v.t.size() / 2], mn = v.t[0];
    printf("{\"variant\":\"%s\",\"median_us\":%.2f,\"min_us\":%.2f,\"GBps\":%.1f}\n", v.name.c_str(), med * 1e3,
           mn * 1e3, v.bytes > 0 ? v.bytes / (med * 1e-3) / 1e9 : 0.0);
  }
  return 0;
}
