// tlbprobe.hip -- streaming read / write / encode-pattern rate vs footprint on MI355X: does a sweep
// over tens of GB run at the rate of a 1-GB sweep?  (Large FEC batches, see
// DESIGN_HISTORY.md §4 "batch size".)  Read-only nt stream, one 16-B chunk per thread,
// full grid, each footprint swept repeatedly after 200 ms of warm load.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/tlbprobe tools/tlbprobe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
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

// Linear forms are grid-stride (a grid stays below 2^32 threads).
constexpr uint32_t kLinBlocks = 1u << 20;

__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ a, uint32_t* out, uint64_t n) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += 256ull * gridDim.x) {
    const u32x4 v = __builtin_nontemporal_load(&a[i]);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = 1u;
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

// Linear nt store stream (write-side translation).
__global__ __launch_bounds__(256) void k_write(u32x4* __restrict__ a, uint64_t n) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += 256ull * gridDim.x) {
    const uint32_t x = static_cast<uint32_t>(i);
    __builtin_nontemporal_store(u32x4{x, x, x, x}, &a[i]);
  }
}

// The (10,3) encode's streams without the arithmetic: 13 rows 1/13 of the
// footprint apart, thread c reads chunk c of rows 0-9 and writes chunk c of
// rows 10-12 (XORs of the inputs), nt loads and stores.
__global__ __launch_bounds__(256) void k_r10w3(uint8_t* __restrict__ a, uint64_t chunks, uint64_t rstride) {
  const uint64_t c = blockIdx.x * 256ull + threadIdx.x;
  if (c >= chunks) return;
  u32x4 x[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) x[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a + k * rstride + c * 16));
  u32x4 y0 = x[0] ^ x[3] ^ x[6] ^ x[9], y1 = x[1] ^ x[4] ^ x[7], y2 = x[2] ^ x[5] ^ x[8];
  __builtin_nontemporal_store(y0, reinterpret_cast<u32x4*>(a + 10 * rstride + c * 16));
  __builtin_nontemporal_store(y1, reinterpret_cast<u32x4*>(a + 11 * rstride + c * 16));
  __builtin_nontemporal_store(y2, reinterpret_cast<u32x4*>(a + 12 * rstride + c * 16));
}

int main(int argc, char** argv) {
  const bool only_slices = argc > 1;
  const uint64_t GB = 1ull << 30;
  const uint64_t maxb = 160 * GB;
  uint8_t* buf;
  uint32_t* out;
  CK(hipMalloc(&buf, maxb));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(buf, 1, maxb));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const char* names[4] = {"linear read", "10 streams, 1/10 apart", "linear nt write", "10 read + 3 write streams, 1/13 apart"};
  for (uint64_t gb : {1ull, 4ull, 16ull, 64ull, 128ull}) {
    if (only_slices) break;
    for (int form = 0; form < 4; ++form) {
      const uint64_t bytes = gb * GB;
      const uint64_t n16 = bytes / 16;
      const uint64_t rstride = bytes / (form == 3 ? 13 : 10) / 4096 * 4096;
      const uint64_t chunks = rstride / 16;
      auto go = [&]() {
        if (form == 0)
          hipLaunchKernelGGL(k_read, dim3(std::min<uint64_t>((n16 + 255) / 256, kLinBlocks)), dim3(256), 0, 0,
                             (const u32x4*)buf, out, n16);
        else if (form == 1)
          hipLaunchKernelGGL(k_read10, dim3((chunks + 255) / 256), dim3(256), 0, 0, buf, out, chunks, rstride);
        else if (form == 2)
          hipLaunchKernelGGL(k_write, dim3(std::min<uint64_t>((n16 + 255) / 256, kLinBlocks)), dim3(256), 0, 0,
                             (u32x4*)buf, n16);
        else
          hipLaunchKernelGGL(k_r10w3, dim3((chunks + 255) / 256), dim3(256), 0, 0, buf, chunks, rstride);
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
      CK(hipGetLastError());
      const double moved = (form == 0 || form == 2) ? double(bytes) : double(rstride) * (form == 3 ? 13 : 10);
      printf("{\"form\":\"%s\",\"footprint_GB\":%llu,\"us\":%.1f,\"TBps\":%.3f}\n",
             names[form], (unsigned long long)gb, ms * 1e3 / reps,
             moved / (ms * 1e-3 / reps) / 1e12);
      fflush(stdout);
    }
  }
  // The bench's geometry: 13 rows of G x 1360 B (row stride G * 1360), the
  // encode's streams over two alternating batches (cold, like bench.py), G
  // from the bench's 65,536 groups to BASELINE configs[3]'s 4M on one GPU.
  for (uint64_t G : {65536ull, 262144ull, 1048576ull, 2097152ull, 4194304ull}) {
    if (only_slices && G != 4194304ull) continue;
    const uint64_t rstride = G * 1360, chunks = rstride / 16, batch = 13 * rstride;
    if (2 * batch > maxb) break;
    int flip = 0;
    auto go = [&]() {
      hipLaunchKernelGGL(k_r10w3, dim3((chunks + 255) / 256), dim3(256), 0, 0, buf + (flip++ & 1) * batch, chunks,
                         rstride);
    };
    auto t0 = std::chrono::steady_clock::now();
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 0.2) {
      go();
      CK(hipDeviceSynchronize());
    }
    const int reps = G >= 1048576 ? 6 : 40;
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) go();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipGetLastError());
    printf("{\"form\":\"encode streams, bench geometry, 2 batches\",\"groups\":%llu,\"batch_GB\":%.2f,\"us\":%.1f,"
           "\"TBps\":%.3f}\n", (unsigned long long)G, batch / 1e9, ms * 1e3 / reps,
           double(rstride) * 13 / (ms * 1e-3 / reps) / 1e12);
    fflush(stdout);
  }
  // The 4M-group geometry processed in slices of consecutive groups (one launch
  // per slice, each covering 1/k of every row): does a slice behave like the
  // smaller batch or like the 4M one?
  {
    const uint64_t G = 4194304ull, rstride = G * 1360, batch = 13 * rstride;
    for (uint64_t slices : {1ull, 4ull, 16ull}) {
      const uint64_t sc = rstride / 16 / slices;  // chunks per slice (per row)
      int flip = 0;
      auto go = [&]() {
        uint8_t* b = buf + (flip++ & 1) * batch;
        for (uint64_t s2 = 0; s2 < slices; ++s2)
          hipLaunchKernelGGL(k_r10w3, dim3((sc + 255) / 256), dim3(256), 0, 0, b + s2 * sc * 16, sc, rstride);
      };
      auto t0 = std::chrono::steady_clock::now();
      while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < 0.2) {
        go();
        CK(hipDeviceSynchronize());
      }
      const int reps = 6;
      CK(hipEventRecord(e0));
      for (int r = 0; r < reps; ++r) go();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      CK(hipGetLastError());
      printf("{\"form\":\"encode streams, 4M-group geometry in slices\",\"slices\":%llu,\"us\":%.1f,\"TBps\":%.3f}\n",
             (unsigned long long)slices, ms * 1e3 / reps, double(rstride) * 13 / (ms * 1e-3 / reps) / 1e12);
      fflush(stdout);
    }
  }
  return 0;
}
