// Probe: can the host store into device memory directly (large BAR), and how
// fast does a resident wave see it?  Allocations tried: hipExtMallocWithFlags
// fine-grained and uncached.  Prints one JSON line per allocation kind.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>

__global__ void k_echo(volatile uint32_t* req, volatile uint32_t* ack, uint32_t n, uint64_t tmo) {
  // one lane: wait for req == i, answer ack = i, n times (bounded by tmo ticks each)
  if (threadIdx.x) return;
  for (uint32_t i = 1; i <= n; ++i) {
    const uint64_t t0 = wall_clock64();
    while (__hip_atomic_load(const_cast<uint32_t*>(req), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != i) {
      if (static_cast<uint64_t>(wall_clock64()) - t0 > tmo) return;
      __builtin_amdgcn_s_sleep(1);
    }
    __hip_atomic_store(const_cast<uint32_t*>(ack), i, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static void run(const char* kind, uint32_t* req_host, uint32_t* req_dev, uint32_t* ack_host, uint32_t* ack_dev) {
  const uint32_t n = 2000;
  *req_host = 0;
  *ack_host = 0;
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipLaunchKernelGGL(k_echo, dim3(1), dim3(64), 0, s, req_dev, ack_dev, n, 100000000ull);  // 1 s per step max
  double tot = 0, best = 1e9;
  bool ok = true;
  for (uint32_t i = 1; i <= n && ok; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    __atomic_store_n(req_host, i, __ATOMIC_RELEASE);
    while (__atomic_load_n(ack_host, __ATOMIC_ACQUIRE) != i) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) { ok = false; break; }
    }
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    if (i > 100) { tot += us; if (us < best) best = us; }
  }
  (void)hipStreamSynchronize(s);
  std::printf("{\"mailbox\": \"%s\", \"ok\": %s, \"round_trip_mean_us\": %.3f, \"min_us\": %.3f}\n", kind,
              ok ? "true" : "false", tot / (n - 100), best);
  std::fflush(stdout);
  (void)hipStreamDestroy(s);
}

int main() {
  // 1. both words in coherent pinned host memory (the production service)
  uint32_t* h = nullptr;
  if (hipHostMalloc(&h, 256, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return 1;
  uint32_t* hd = nullptr;
  (void)hipHostGetDevicePointer(reinterpret_cast<void**>(&hd), h, 0);
  run("host_coherent", h, hd, h + 32, hd + 32);
  // 2. request word in fine-grained device memory written by the host, ack in host memory
  uint32_t* d = nullptr;
  if (hipExtMallocWithFlags(reinterpret_cast<void**>(&d), 4096, hipDeviceMallocFinegrained) == hipSuccess) {
    hipPointerAttribute_t at{};
    (void)hipPointerGetAttributes(&at, d);
    std::printf("{\"finegrained_attr\": {\"type\": %d, \"hostPointer\": %p, \"devicePointer\": %p}}\n",
                static_cast<int>(at.type), at.hostPointer, at.devicePointer);
    std::fflush(stdout);
    uint32_t* dh = static_cast<uint32_t*>(at.hostPointer ? at.hostPointer : d);
    dh[0] = 7;  // host store into device memory: segfaults if not host-mapped
    std::printf("{\"host_store_into_device_memory\": %u}\n", dh[0]);
    std::fflush(stdout);
    run("device_finegrained_req", dh, d, h + 32, hd + 32);
  }
  return 0;
}
