// layout_probe.hip -- which batch layout gives the (10,3) encode's access
// pattern the highest HBM rate?  The compute-free encode twin (k_encode_g's
// grid, 13-row LDS stage with rows 0-7 by LDS-DMA, 3 blocks per CU, nt loads
// and stores; XOR instead of the GF network) with the data rows and the parity
// rows addressed separately:
//   data row k of group g   at dbase + g * dgs + k * drs
//   parity row i of group g at pbase + g * pgs + i * prs
// Layouts (65,536 groups, pitch 1360, S = 1350), cold regime (3 rotated sets,
// a cache-evicting sweep before every sample), interleaved, medians.  Also the
// one-chunk-per-thread nt copy of the same bytes.  Not product code.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iugo_amd/csrc -o tools/layout_probe tools/layout_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "gf_device.hpp"

using namespace ugo::kern;

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

struct L {
  const uint8_t* d;
  uint8_t* p;
  uint64_t drs, dgs, prs, pgs;
  uint32_t chunks, S, items;
};

template <int GR>
__global__ __launch_bounds__(256) void k_twin(L a) {
  constexpr int D = 10, P = 3, LR = 13;
  __shared__ u32x4 stage[4][LR][64];
  const uint32_t item = blockIdx.x * 256u + threadIdx.x;
  if (item >= a.items) return;
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t gl = item / a.chunks, c = item - gl * a.chunks;
  const uint8_t* dp = a.d + gl * a.dgs + static_cast<uint64_t>(c) * 16u;
  uint8_t* pp = a.p + gl * a.pgs + static_cast<uint64_t>(c) * 16u;
  const uint32_t nb = a.S - c * 16u;
#pragma unroll
  for (int k = 0; k < GR; ++k) lds_dma16(dp + static_cast<uint64_t>(k) * a.drs, &stage[w][k][0]);
  V4 x[D];
#pragma unroll
  for (int k = GR; k < D; ++k) x[k] = load16<1>(dp + static_cast<uint64_t>(k) * a.drs);
  if (GR) lds_dma_wait();
#pragma unroll
  for (int k = 0; k < GR; ++k) x[k] = lds16(&stage[w][k][lane]);
#pragma unroll
  for (int i = 0; i < P; ++i) {
    V4 y = x[i];
#pragma unroll
    for (int k = 0; k < D; ++k)
      if (k != i)
#pragma unroll
        for (int j = 0; j < 4; ++j) y.v[j] ^= x[k].v[j];
    store16<2>(pp + static_cast<uint64_t>(i) * a.prs, y, nb);
  }
}

__global__ __launch_bounds__(256) void k_copy1(const u32x4* src, u32x4* dst, uint64_t n16) {
  const uint64_t c = blockIdx.x * 256ull + threadIdx.x;
  if (c >= n16) return;
  __builtin_nontemporal_store(__builtin_nontemporal_load(src + c), dst + c);
}

__global__ __launch_bounds__(256) void k_flush(const u32x4* a, uint32_t* out, uint64_t n16) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i >= n16) return;
  const u32x4 v = a[i];
  if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9e3779b9u) out[0] = v.x;
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 15;
  const uint64_t G = 65536, pitch = 1360, S = 1350, chunks = (S + 15) / 16;
  const uint64_t bytes_set = G * 13 * pitch;
  std::vector<uint8_t*> sets(3);
  for (auto& b : sets) {
    CK(hipMalloc(&b, bytes_set + 4096));
    CK(hipMemset(b, 0x5a, bytes_set + 4096));
  }
  struct Layout {
    std::string name;
    uint64_t drs, dgs, prs, pgs, poff;  // parity base = set + poff
  };
  const std::vector<Layout> lays = {
      {"planar [13][G][pitch] (production)", G * pitch, pitch, G * pitch, pitch, 10 * G * pitch},
      {"data group-major [G][10][pitch] + parity planar [3][G][pitch]", pitch, 10 * pitch, G * pitch, pitch,
       10 * G * pitch},
      {"data group-major [G][10][pitch] + parity group-major [G][3][pitch]", pitch, 10 * pitch, pitch, 3 * pitch,
       10 * G * pitch},
      {"group-major [G][13][pitch]", pitch, 13 * pitch, pitch, 13 * pitch, 10 * pitch},
      {"data planar + parity group-major [G][3][pitch]", G * pitch, pitch, pitch, 3 * pitch, 10 * G * pitch},
  };
  const uint32_t items = static_cast<uint32_t>(G * chunks);
  const uint32_t blocks = (items + 255) / 256;
  struct T {
    std::string name;
    std::function<void(int)> fn;
    std::vector<float> t;
  };
  std::vector<T> ts;
  for (const auto& l : lays) {
    for (int gr : {8, 0}) {
      ts.push_back({l.name + (gr ? ", 8 rows by LDS-DMA" : ", all rows by nt register loads"), [&, l, gr](int k) {
                      L a{sets[k], sets[k] + l.poff, l.drs, l.dgs, l.prs, l.pgs, static_cast<uint32_t>(chunks),
                          static_cast<uint32_t>(S), items};
                      if (gr)  // the 52-KiB static stage: 3 blocks per CU
                        k_twin<8><<<blocks, 256, 0>>>(a);
                      else  // no stage: the same 3 blocks per CU held by unused dynamic LDS
                        k_twin<0><<<blocks, 256, 13u * 4u * 64u * 16u>>>(a);
                    }, {}});
    }
  }
  const uint64_t enc_bytes = G * 13 * S;
  const uint64_t copy16 = enc_bytes / 2 / 16;
  ts.push_back({"nt copy of the same bytes", [&](int k) {
                  k_copy1<<<(copy16 + 255) / 256, 256>>>(reinterpret_cast<const u32x4*>(sets[k]),
                                                         reinterpret_cast<u32x4*>(sets[k] + bytes_set / 2), copy16);
                }, {}});
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int cnt = 0;
  for (int w = 0; w < 4; ++w)
    for (auto& v : ts) v.fn(cnt++ % 3);
  CK(hipDeviceSynchronize());
  const uint64_t fl16 = (768ull << 20) / 16;
  uint8_t* fl = nullptr;
  CK(hipMalloc(&fl, fl16 * 16));
  CK(hipMemset(fl, 1, fl16 * 16));
  for (int rr = 0; rr < rounds; ++rr)
    for (auto& v : ts) {
      k_flush<<<(fl16 + 255) / 256, 256>>>(reinterpret_cast<const u32x4*>(fl), reinterpret_cast<uint32_t*>(fl), fl16);
      CK(hipEventRecord(e0));
      for (int k = 0; k < 3; ++k) v.fn(cnt++ % 3);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.t.push_back(ms * 1000.f / 3.f);
    }
  CK(hipGetLastError());
  for (auto& v : ts) {
    std::sort(v.t.begin(), v.t.end());
    const double med = v.t[v.t.size() / 2];
    printf("{\"variant\":\"%s\",\"median_us\":%.2f,\"min_us\":%.2f,\"GBps\":%.1f,\"frac\":%.4f}\n", v.name.c_str(), med,
           v.t[0], enc_bytes / med / 1e3, enc_bytes / med / 1e3 / 8000.0);
  }
  return 0;
}
