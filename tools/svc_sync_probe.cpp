// svc_sync_probe.cpp -- which HIP calls wait for a resident per-call service
// block (k_service polls its mailbox until idle_us without a request)?  The
// bench's interference A/B found ugo_fec_encode_host of 65,536 groups taking
// ~1 s (the idle window) instead of ~17 ms while a service block was resident
// on another context.  Each call below is timed with and without a resident
// block (idle window 1 s, one served call just before).  Not product code.
// Build: hipcc -O2 -std=c++17 -o tools/svc_sync_probe tools/svc_sync_probe.cpp -Lugo_amd -lugofec -Wl,-rpath,'$ORIGIN/../ugo_amd'
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../include/ugo_fec.h"

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

static double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

int main() {
  const int d = 10, p = 3, n = 13;
  const size_t S = 1350, pitch = 1360, G = 8192, gbytes = n * pitch;
  ugo_fec* svc = nullptr;
  ugo_fec* work = nullptr;
  if (ugo_fec_create(0, d, p, &svc) || ugo_fec_create(0, d, p, &work)) return 1;
  uint8_t* one = nullptr;
  uint8_t* host = nullptr;
  if (ugo_fec_host_alloc(n * 1472, reinterpret_cast<void**>(&one)) ||
      ugo_fec_host_alloc(G * gbytes, reinterpret_cast<void**>(&host)))
    return 1;
  std::memset(one, 1, n * 1472);
  std::memset(host, 2, G * gbytes);
  uint8_t* dev = nullptr;
  CK(hipMalloc(&dev, G * gbytes));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  struct Op {
    std::string name;
    std::function<int()> fn;
  };
  std::vector<Op> ops = {
      {"hipMemcpyAsync H2D pinned 106 MB + stream sync", [&] {
         CK(hipMemcpyAsync(dev, host, G * gbytes, hipMemcpyHostToDevice, s));
         CK(hipStreamSynchronize(s));
         return 0;
       }},
      {"hipMemcpy2DAsync H2D pinned (data rows) + stream sync", [&] {
         CK(hipMemcpy2DAsync(dev, gbytes, host, gbytes, d * pitch, G, hipMemcpyHostToDevice, s));
         CK(hipStreamSynchronize(s));
         return 0;
       }},
      {"hipMemcpy3DAsync D2H pinned (parity rows, [0,S)) + stream sync", [&] {
         hipMemcpy3DParms cp{};
         cp.srcPtr = make_hipPitchedPtr(dev, pitch, pitch, n);
         cp.srcPos = make_hipPos(0, d, 0);
         cp.dstPtr = make_hipPitchedPtr(host, pitch, pitch, n);
         cp.dstPos = make_hipPos(0, d, 0);
         cp.extent = make_hipExtent(S, p, G);
         cp.kind = hipMemcpyDeviceToHost;
         CK(hipMemcpy3DAsync(&cp, s));
         CK(hipStreamSynchronize(s));
         return 0;
       }},
      {"ugo_fec_encode (device batch) + stream sync", [&] {
         if (ugo_fec_encode(work, dev, G, S, pitch, s)) return 1;
         CK(hipStreamSynchronize(s));
         return 0;
       }},
      {"ugo_fec_encode_host (pinned, staged pipeline)", [&] { return ugo_fec_encode_host(work, host, G, S, pitch); }},
      {"hipMemsetAsync 4 B on the null stream + its sync", [&] {
         CK(hipMemsetAsync(dev, 0, 4, nullptr));
         CK(hipStreamSynchronize(nullptr));
         return 0;
       }},
      {"hipMemsetAsync 4 B on each of 8 fresh streams + sync (ms = worst stream)", [&] {
         double worst = 0;
         for (int i = 0; i < 8; ++i) {
           hipStream_t t;
           CK(hipStreamCreateWithFlags(&t, hipStreamNonBlocking));
           const auto t0 = std::chrono::steady_clock::now();
           CK(hipMemsetAsync(dev, 0, 4, t));
           CK(hipStreamSynchronize(t));
           worst = std::max(worst, ms_since(t0));
           CK(hipStreamDestroy(t));
         }
         return worst > 100 ? 2 : 0;  // rc 2: some stream queued behind the block
       }},
      {"hipMalloc + hipFree 1 MB", [&] {
         void* q = nullptr;
         CK(hipMalloc(&q, 1 << 20));
         CK(hipFree(q));
         return 0;
       }},
  };
  for (int round = 0; round < 2; ++round)
    for (int mode = 0; mode < 2; ++mode) {
      if (mode == 1) {
        if (ugo_fec_service_start(svc, 1000000)) return 1;
        if (ugo_fec_encode_host(svc, one, 1, 1470, 1472)) return 1;  // served: the block is resident now
      }
      for (auto& op : ops) {
        const auto t0 = std::chrono::steady_clock::now();
        const int rc = op.fn();
        printf("{\"round\":%d,\"service_resident\":%s,\"op\":\"%s\",\"rc\":%d,\"ms\":%.3f}\n", round,
               mode ? "true" : "false", op.name.c_str(), rc, ms_since(t0));
        fflush(stdout);
        if (mode == 1 && ugo_fec_encode_host(svc, one, 1, 1470, 1472)) return 1;  // keep it resident
      }
      if (mode == 1 && ugo_fec_service_stop(svc)) return 1;
    }
  ugo_fec_host_free(one);
  ugo_fec_host_free(host);
  (void)hipFree(dev);
  ugo_fec_destroy(svc);
  ugo_fec_destroy(work);
  return 0;
}
