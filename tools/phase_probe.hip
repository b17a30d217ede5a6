// phase_probe.hip -- does grouping the encode's writes into bursts move its
// mixed read/write ceiling?  The (10,3) encode's streams without the
// arithmetic (10 nt row reads, 3 nt row writes per 16-B chunk, XOR as the
// "parity") at the bench geometry (65,536 groups x 1360 B per row, two
// alternating batches, so every launch is cache-cold like bench.py):
//   base        one chunk per thread, full grid (tlbprobe's k_r10w3)
//   burst K     a thread reads K chunks of every data row, holding K x 3
//               parity chunks in registers, then writes them all: each wave
//               alternates a read phase of K x 10 KiB and a write phase of
//               K x 3 KiB (full grid)
//   persist K/B the same tiles on a persistent grid of B blocks per CU, so
//               the blocks start their phases together and, with equal work,
//               stay roughly in step chip-wide (no grid barrier)
// The question is DESIGN_HISTORY.md §8.1's: a 10-read + 3-write mix runs at 6.0 TB/s
// where 10 read streams alone run at 6.9 and one write stream at 6.8
// (profiles/r2/tlbprobe_r2.jsonl).  Not product code.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/phase_probe tools/phase_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

__device__ __forceinline__ u32x4 ld(const uint8_t* p) { return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p)); }
__device__ __forceinline__ void st(uint8_t* p, u32x4 v) { __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p)); }

__global__ __launch_bounds__(256) void k_base(uint8_t* __restrict__ a, uint64_t chunks, uint64_t rstride) {
  const uint64_t c = blockIdx.x * 256ull + threadIdx.x;
  if (c >= chunks) return;
  u32x4 x[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) x[k] = ld(a + k * rstride + c * 16);
  st(a + 10 * rstride + c * 16, x[0] ^ x[3] ^ x[6] ^ x[9]);
  st(a + 11 * rstride + c * 16, x[1] ^ x[4] ^ x[7]);
  st(a + 12 * rstride + c * 16, x[2] ^ x[5] ^ x[8]);
}

// One tile = K x 256 consecutive chunks of every row; thread t takes chunks
// tile*K*256 + j*256 + t, j < K (each wave instruction: 1 KiB contiguous).
template <int K>
__device__ __forceinline__ void tile(uint8_t* __restrict__ a, uint64_t t, uint64_t rstride) {
  u32x4 y[K][3];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const uint64_t off = ((t * K + j) * 256ull + threadIdx.x) * 16;
    u32x4 x[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) x[k] = ld(a + k * rstride + off);
    y[j][0] = x[0] ^ x[3] ^ x[6] ^ x[9];
    y[j][1] = x[1] ^ x[4] ^ x[7];
    y[j][2] = x[2] ^ x[5] ^ x[8];
  }
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < K; ++j) st(a + (10 + i) * rstride + ((t * K + j) * 256ull + threadIdx.x) * 16, y[j][i]);
}

template <int K>
__global__ __launch_bounds__(256) void k_burst(uint8_t* __restrict__ a, uint64_t tiles, uint64_t rstride) {
  if (blockIdx.x < tiles) tile<K>(a, blockIdx.x, rstride);
}

template <int K>
__global__ __launch_bounds__(256) void k_persist(uint8_t* __restrict__ a, uint64_t tiles, uint64_t rstride) {
  for (uint64_t t = blockIdx.x; t < tiles; t += gridDim.x) tile<K>(a, t, rstride);
}

int main() {
  const uint64_t G = 65536, pitch = 1360, rstride = G * pitch, chunks = rstride / 16, batch = 13 * rstride;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint8_t* buf;
  CK(hipMalloc(&buf, 2 * batch));
  CK(hipMemset(buf, 1, 2 * batch));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct V {
    const char* name;
    int K, bpc;  // bpc = 0: full grid
  };
  const std::vector<V> vs = {{"base", 1, 0},      {"burst", 2, 0},    {"burst", 4, 0},    {"burst", 8, 0},
                             {"persist", 2, 2},   {"persist", 2, 4},  {"persist", 4, 2},  {"persist", 4, 3},
                             {"persist", 8, 1},   {"persist", 8, 2},  {"persist", 1, 4},  {"persist", 1, 8}};
  int flip = 0;
  auto launch = [&](const V& v) {
    uint8_t* b = buf + (flip++ & 1) * batch;
    const uint64_t tiles = chunks / (256ull * v.K);
    const dim3 grid = v.bpc ? dim3(cus * v.bpc) : dim3(tiles);
    if (v.bpc == 0) {
      if (v.K == 1) hipLaunchKernelGGL(k_base, dim3(chunks / 256), dim3(256), 0, 0, b, chunks, rstride);
      if (v.K == 2) hipLaunchKernelGGL(k_burst<2>, grid, dim3(256), 0, 0, b, tiles, rstride);
      if (v.K == 4) hipLaunchKernelGGL(k_burst<4>, grid, dim3(256), 0, 0, b, tiles, rstride);
      if (v.K == 8) hipLaunchKernelGGL(k_burst<8>, grid, dim3(256), 0, 0, b, tiles, rstride);
    } else {
      if (v.K == 1) hipLaunchKernelGGL(k_persist<1>, grid, dim3(256), 0, 0, b, tiles, rstride);
      if (v.K == 2) hipLaunchKernelGGL(k_persist<2>, grid, dim3(256), 0, 0, b, tiles, rstride);
      if (v.K == 4) hipLaunchKernelGGL(k_persist<4>, grid, dim3(256), 0, 0, b, tiles, rstride);
      if (v.K == 8) hipLaunchKernelGGL(k_persist<8>, grid, dim3(256), 0, 0, b, tiles, rstride);
    }
  };
  // clock warm-up
  auto t0 = std::chrono::steady_clock::now();
  while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 0.3) {
    launch(vs[0]);
    CK(hipDeviceSynchronize());
  }
  const int rounds = 7, reps = 20;
  std::vector<std::vector<float>> us(vs.size());
  for (int r = 0; r < rounds; ++r)
    for (size_t i = 0; i < vs.size(); ++i) {
      for (int w = 0; w < 4; ++w) launch(vs[i]);
      CK(hipEventRecord(e0));
      for (int q = 0; q < reps; ++q) launch(vs[i]);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      CK(hipGetLastError());
      us[i].push_back(ms * 1e3f / reps);
    }
  for (size_t i = 0; i < vs.size(); ++i) {
    std::sort(us[i].begin(), us[i].end());
    const double med = us[i][rounds / 2];
    printf("{\"variant\":\"%s\",\"K\":%d,\"blocks_per_cu\":%d,\"us_median\":%.1f,\"us_min\":%.1f,\"TBps\":%.3f}\n",
           vs[i].name, vs[i].K, vs[i].bpc, med, us[i][0], double(13 * rstride) / (med * 1e-6) / 1e12);
  }
  return 0;
}
