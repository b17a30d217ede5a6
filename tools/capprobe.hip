// capprobe.hip -- residency caps of the (10,3) kernels by batch size
// (VERDICT r2 item 1): interleaved A/B of the production encode and
// reconstruct_into at 2/3/4/5 blocks per CU, on a batch of G groups.
// Usage: capprobe G rounds [row_pad] [nbuf]: row_pad bytes added to the planar
// row stride (G * pitch + row_pad).  G >= 1M: one batch (its 18+ GB are far past the
// 256-MB Infinity Cache, so every launch is cold); G < 1M: 4 rotating
// batches, as kvariants' cold regime.  Prints one JSON line per variant
// (median us, TB/s of algorithmic bytes).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/capprobe tools/capprobe.hip
// Not product code: it includes the kernel TU to instantiate the variants.
#include "../ugo_amd/csrc/fec_kernels.hip"

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

int main(int argc, char** argv) {
  const int d = 10, p = 3, n = 13;
  const uint32_t S = 1350, pitch = 1360;
  const uint64_t G = argc > 1 ? atoll(argv[1]) : 4194304;
  const int rounds = argc > 2 ? atoi(argv[2]) : 9;
  const int nb = G >= (1u << 20) ? 1 : 4;
  const uint64_t row_pad = argc > 3 ? atoll(argv[3]) : 0;
  const uint64_t rstride = G * pitch + row_pad;
  std::vector<Batch> rot(nb), roto(nb);
  uint64_t* masks;
  CK(hipMalloc(&masks, G * 8));
  {
    std::vector<uint64_t> hm(G);
    uint64_t st = 0x5EED;
    for (uint64_t g = 0; g < G; ++g) {
      st = st * 6364136223846793005ull + 1442695040888963407ull;
      int a = (st >> 33) % n, b = (a + 1 + (st >> 40) % (n - 1)) % n;
      hm[g] = ((1ull << n) - 1) & ~(1ull << a) & ~(1ull << b);
    }
    CK(hipMemcpy(masks, hm.data(), G * 8, hipMemcpyHostToDevice));
  }
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
  for (int r = 0; r < nb; ++r) {
    uint8_t *buf, *ob;
    CK(hipMalloc(&buf, n * rstride));
    CK(hipMalloc(&ob, p * rstride));
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, buf, n * rstride / 16, 77ull + r);
    Batch a{};
    a.mult = dmul;
    a.base = buf; a.gstride = pitch; a.rstride = rstride; a.nmask = (1ull << n) - 1; a.S = S;
    a.chunks = 85; a.items = static_cast<uint32_t>(G * 85); a.desc = dtab; a.present = masks;
    a.desc_stride = stride; a.d = d; a.dpad = dpad; a.epad = epad;
    rot[r] = a;
    a.out = ob; a.ogstride = pitch; a.orstride = rstride;
    roto[r] = a;
  }
  CK(hipDeviceSynchronize());
  const double enc_bytes = double(G) * n * S, dec_bytes = double(G) * 12 * S;
  const uint32_t grid = static_cast<uint32_t>((G * 85 + 255) / 256);
  auto extra = [](uint32_t bpc, uint32_t static_b) { return 160u * 1024u / bpc - static_b - 1024u; };
  struct Var { std::string name; double bytes; std::function<void(int)> go; std::vector<float> t; };
  std::vector<Var> vars;
  // k_encode_g<10,3,2,8,256,LR>: LR-row stage, LR * 4 KiB static LDS per block
  vars.push_back({"enc 13-row stage (3 blocks/CU, production)", enc_bytes, [&](int r) {
    hipLaunchKernelGGL((k_encode_g<10, 3, 2, 8, 256, 13>), dim3(grid), dim3(256), 0, 0, rot[r]); }, {}});
  for (uint32_t bpc : {5u, 4u, 2u}) {
    const uint32_t x = bpc == 5 ? 0u : extra(bpc, 32u * 1024u);
    vars.push_back({"enc 8-row stage, " + std::to_string(bpc) + " blocks/CU", enc_bytes, [&, x](int r) {
      hipLaunchKernelGGL((k_encode_g<10, 3, 2, 8, 256, 8>), dim3(grid), dim3(256), x, 0, rot[r]); }, {}});
  }
  vars.push_back({"enc 8-row stage, 3 blocks/CU (dyn LDS)", enc_bytes, [&](int r) {
    hipLaunchKernelGGL((k_encode_g<10, 3, 2, 8, 256, 8>), dim3(grid), dim3(256), extra(3, 32u * 1024u), 0, rot[r]); }, {}});
  for (uint32_t bpc : {5u, 4u, 3u, 2u}) {  // k_apply_p: no static LDS, 99 VGPRs: 5 waves/SIMD natively
    const uint32_t x = bpc == 5 ? 0u : extra(bpc, 0u);
    vars.push_back({"dec into k_apply_p, " + std::to_string(bpc) + " blocks/CU", dec_bytes, [&, x](int r) {
      hipLaunchKernelGGL((k_apply_p<10, 1, 3>), dim3(grid), dim3(256), x, 0, roto[r]); }, {}});
  }
  // the bench step: encode then reconstruct_into of the same batch, each timed
  // on its own (is a reconstruct right after an encode slower than one after
  // another reconstruct?)
  std::vector<float> step_enc, step_dec;
  hipEvent_t s0, s1, s2;
  CK(hipEventCreate(&s0));
  CK(hipEventCreate(&s1));
  CK(hipEventCreate(&s2));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int cnt = 0;
  for (int w = 0; w < 3; ++w)  // clocks up
    for (auto& v : vars) v.go(cnt++ % nb);
  CK(hipDeviceSynchronize());
  for (int rd = 0; rd < rounds; ++rd) {
    {
      const int r = cnt++ % nb;
      CK(hipEventRecord(s0));
      hipLaunchKernelGGL((k_encode_g<10, 3, 2, 8, 256, 13>), dim3(grid), dim3(256), 0, 0, rot[r]);
      CK(hipEventRecord(s1));
      hipLaunchKernelGGL((k_apply_p<10, 1, 3>), dim3(grid), dim3(256), 0, 0, roto[r]);
      CK(hipEventRecord(s2));
      CK(hipEventSynchronize(s2));
      float a1 = 0, a2 = 0;
      CK(hipEventElapsedTime(&a1, s0, s1));
      CK(hipEventElapsedTime(&a2, s1, s2));
      step_enc.push_back(a1);
      step_dec.push_back(a2);
    }
    for (auto& v : vars) {
      const int r = cnt++ % nb;
      CK(hipEventRecord(e0));
      v.go(r);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.t.push_back(ms);
    }
  }
  // placement: nbuf more batches (inputs + outputs in one allocation each),
  // production encode and reconstruct_into timed on each, back to back
  const int nbuf = argc > 4 ? atoi(argv[4]) : 0;
  for (int b = 0; b < nbuf; ++b) {
    uint8_t* cp;
    if (hipMalloc(&cp, (n + p) * rstride) != hipSuccess) break;
    CK(hipMemcpy(cp, rot[0].base, n * rstride, hipMemcpyDeviceToDevice));
    Batch x = rot[0], y = roto[0];
    x.base = cp; y.base = cp; y.out = cp + n * rstride;
    std::vector<float> te, td;
    for (int r = 0; r < rounds + 3; ++r) {
      CK(hipEventRecord(s0));
      hipLaunchKernelGGL((k_encode_g<10, 3, 2, 8, 256, 13>), dim3(grid), dim3(256), 0, 0, x);
      CK(hipEventRecord(s1));
      hipLaunchKernelGGL((k_apply_p<10, 1, 3>), dim3(grid), dim3(256), 0, 0, y);
      CK(hipEventRecord(s2));
      CK(hipEventSynchronize(s2));
      float a1 = 0, a2 = 0;
      CK(hipEventElapsedTime(&a1, s0, s1));
      CK(hipEventElapsedTime(&a2, s1, s2));
      if (r >= 3) { te.push_back(a1); td.push_back(a2); }
    }
    std::sort(te.begin(), te.end());
    std::sort(td.begin(), td.end());
    printf("{\"G\": %llu, \"row_pad\": %llu, \"buffer\": %d, \"va\": \"%p\", \"enc_median_us\": %.1f, \"dec_median_us\": %.1f}\n",
           (unsigned long long)G, (unsigned long long)row_pad, b + 1, (void*)cp, te[te.size() / 2] * 1e3, td[td.size() / 2] * 1e3);
    fflush(stdout);
  }
  std::sort(step_enc.begin(), step_enc.end());
  std::sort(step_dec.begin(), step_dec.end());
  printf("{\"G\": %llu, \"row_pad\": %llu, \"variant\": \"STEP enc (production) then dec into (production) on the same batch\", "
         "\"enc_median_us\": %.1f, \"dec_median_us\": %.1f, \"enc_TBps\": %.3f, \"dec_TBps\": %.3f}\n",
         (unsigned long long)G, (unsigned long long)row_pad, step_enc[step_enc.size() / 2] * 1e3, step_dec[step_dec.size() / 2] * 1e3,
         enc_bytes / (step_enc[step_enc.size() / 2] * 1e-3) / 1e12, dec_bytes / (step_dec[step_dec.size() / 2] * 1e-3) / 1e12);
  for (auto& v : vars) {
    std::sort(v.t.begin(), v.t.end());
    const double med = v.t[v.t.size() / 2];
    printf("{\"G\": %llu, \"row_pad\": %llu, \"variant\": \"%s\", \"median_us\": %.1f, \"TBps\": %.3f, \"min_us\": %.1f, \"max_us\": %.1f}\n",
           (unsigned long long)G, (unsigned long long)row_pad, v.name.c_str(), med * 1e3, v.bytes / (med * 1e-3) / 1e12, v.t.front() * 1e3,
           v.t.back() * 1e3);
  }
  return 0;
}
