// tlbprobe.hip -- streaming read rate vs footprint on MI355X: does a sweep
// over tens of GB run at the rate of a 1-GB sweep?  (Large FEC batches, see
// DESIGN.md §4 "batch size".)  Read-only nt stream, one 16-B chunk per thread,
// full grid, each footprint swept repeatedly after 200 ms of warm load.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/tlbprobe tools/tlbprobe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ a, uint32_t* out, uint64_t n) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i >= n) return;
  const u32x4 v = __builtin_nontemporal_load(&a[i]);
  if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345678u) out[0] = 1u;
}

// 10 streams 1/10 of the footprint apart, like the data rows of a planar
// batch: thread c reads chunk c of every stream (the encode's loads, no stores).
__global__ __launch_bounds__(256) void k_read10(const uint8_t* __restrict__ a, uint32_t* out, uint64_t chunks,
                                                uint64_t rstride) {
  const uint64_t c = blockIdx.x * 256ull + threadIdx.x;
  if (c >= chunks) return;
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a + k * rstride + c * 16));
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = 1u;
}

int main() {
  const uint64_t GB = 1ull << 30;
  const uint64_t maxb = 64 * GB;
  uint8_t* buf;
  uint32_t* out;
  CK(hipMalloc(&buf, maxb));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(buf, 1, maxb));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (uint64_t gb : {1ull, 4ull, 16ull, 64ull}) {
    for (int form = 0; form < 2; ++form) {
      const uint64_t bytes = gb * GB;
      const uint64_t n16 = bytes / 16;
      const uint64_t rstride = bytes / 10 / 4096 * 4096;
      const uint64_t chunks = rstride / 16;
      auto go = [&]() {
        if (form == 0)
          hipLaunchKernelGGL(k_read, dim3((n16 + 255) / 256), dim3(256), 0, 0, (const u32x4*)buf, out, n16);
        else
          hipLaunchKernelGGL(k_read10, dim3((chunks + 255) / 256), dim3(256), 0, 0, buf, out, chunks, rstride);
      };
      auto t0 = std::chrono::steady_clock::now();
      while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 0.2) {
        go();
        CK(hipDeviceSynchronize());
      }
      const int reps = gb >= 16 ? 5 : 20;
      CK(hipEventRecord(e0));
      for (int r = 0; r < reps; ++r) go();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double moved = form == 0 ? double(bytes) : double(rstride) * 10;
      printf("{\"form\":\"%s\",\"footprint_GB\":%llu,\"us\":%.1f,\"TBps\":%.3f}\n",
             form == 0 ? "linear read" : "10 streams, 1/10 apart", (unsigned long long)gb, ms * 1e3 / reps,
             moved / (ms * 1e-3 / reps) / 1e12);
      fflush(stdout);
    }
  }
  return 0;
}
