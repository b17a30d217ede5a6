// svc_stage_probe.hip -- VERDICT r4 item 6, bounded A/B of the per-call
// service's input path: the block reads a request's d rows (10 x 1472 B, one
// (10,3) group) over PCIe from pinned host memory (production), against the
// host first writing those rows into device memory it can map (fine-grained
// device memory, write-combined over the large BAR, then sfence) and the block
// reading them from HBM.  Measured: the block's own read time (wall_clock64
// around its loads, one 512-thread block as k_service), and the host's write +
// fence time; many repetitions, medians.  Not product code.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -Xarch_host -mavx2 -o tools/svc_stage_probe tools/svc_stage_probe.hip
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// one block of 512 threads: every thread loads its share of the rows' 16-B
// chunks (10 rows x 92 chunks = 920 loads, <= 2 per thread), then the block
// waits for all of them; ticks[0] = the read's duration in wall-clock ticks
__global__ __launch_bounds__(512) void k_read_rows(const uint8_t* src, uint32_t rows, uint32_t pitch, uint32_t chunks,
                                                   uint64_t* ticks, uint32_t* sink) {
  __syncthreads();
  const uint64_t t0 = wall_clock64();
  u32x4 acc = {0u, 0u, 0u, 0u};
  for (uint32_t i = threadIdx.x; i < rows * chunks; i += 512u) {
    const uint32_t r = i / chunks, c = i - r * chunks;
    acc ^= *reinterpret_cast<const volatile u32x4*>(src + uint64_t(r) * pitch + 16u * c);
  }
  __syncthreads();
  const uint64_t t1 = wall_clock64();
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x9e3779b9u) sink[0] = acc.x;
  if (threadIdx.x == 0) ticks[0] = t1 - t0;
}

int main() {
  const uint32_t rows = 10, pitch = 1472, chunks = 92, bytes = rows * pitch;
  int khz = 100000;
  (void)hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0);
  uint8_t *pinned = nullptr, *stage = nullptr, *dstage = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&pinned), bytes, hipHostMallocCoherent | hipHostMallocMapped));
  for (uint32_t i = 0; i < bytes; ++i) pinned[i] = static_cast<uint8_t>(i * 7);
  CK(hipExtMallocWithFlags(reinterpret_cast<void**>(&dstage), bytes, hipDeviceMallocFinegrained));
  hipPointerAttribute_t at{};
  CK(hipPointerGetAttributes(&at, dstage));
  stage = static_cast<uint8_t*>(at.hostPointer);
  printf("{\"stage\":\"fine-grained device memory\",\"type\":%d,\"host_pointer\":%s}\n", static_cast<int>(at.type),
         stage ? "true" : "false");
  uint64_t* ticks;
  uint32_t* sink;
  CK(hipMalloc(&ticks, 8));
  CK(hipMalloc(&sink, 4));
  uint8_t* dpinned = nullptr;
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dpinned), pinned, 0));
  auto read_us = [&](const uint8_t* src, std::vector<double>& out) -> int {
    for (int r = 0; r < 203; ++r) {
      k_read_rows<<<1, 512>>>(src, rows, pitch, chunks, ticks, sink);
      CK(hipDeviceSynchronize());
      uint64_t t = 0;
      CK(hipMemcpy(&t, ticks, 8, hipMemcpyDeviceToHost));
      if (r >= 3) out.push_back(double(t) * 1000.0 / khz);
    }
    return 0;
  };
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  std::vector<double> tp, td, tw;
  if (read_us(dpinned, tp)) return 1;
  if (read_us(dstage, td)) return 1;
  if (stage) {  // the host's side: write the rows into the mapped device memory, fence
    for (int r = 0; r < 2003; ++r) {
      const auto t0 = std::chrono::steady_clock::now();
      for (uint32_t i = 0; i < bytes; i += 64) {
        const __m256i* s = reinterpret_cast<const __m256i*>(pinned + i);
        _mm256_stream_si256(reinterpret_cast<__m256i*>(stage + i), _mm256_loadu_si256(s));
        if (i + 32 < bytes) _mm256_stream_si256(reinterpret_cast<__m256i*>(stage + i + 32), _mm256_loadu_si256(s + 1));
      }
      _mm_sfence();
      const auto t1 = std::chrono::steady_clock::now();
      if (r >= 3) tw.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    std::vector<uint8_t> back(bytes);
    CK(hipMemcpy(back.data(), dstage, bytes, hipMemcpyDeviceToHost));
    printf("{\"check\":\"staged rows equal the source\",\"equal\":%s}\n",
           std::memcmp(back.data(), pinned, bytes) == 0 ? "true" : "false");
  }
  printf("{\"block_read_us_pinned_pcie\":%.3f,\"block_read_us_device_hbm\":%.3f,\"host_write_fence_us\":%s,"
         "\"bytes\":%u}\n",
         med(tp), med(td), stage ? std::to_string(med(tw)).c_str() : "null", bytes);
  return 0;
}
