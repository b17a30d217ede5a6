// launch_floor.hip -- the per-call floor of the drop-in path on MI355X: one
// tiny kernel launch + one synchronize, the shape of every per-group call
// (DESIGN_HISTORY.md §4 "drop-in per-group path").  Variants: default device flags vs
// hipDeviceScheduleSpin, stream synchronize vs event synchronize, and a
// kernel that touches a pinned (mapped) host buffer like the zero-copy calls.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/launch_floor tools/launch_floor.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

__global__ void k_empty() {}

// one group of (10+3)x1360 B through a mapped pointer: each of 85 lanes reads
// 10 chunks and writes 3 (no arithmetic), like the zero-copy encode of G = 1
__global__ void k_touch(uint4* g, int chunks, int rstride16) {
  const int c = threadIdx.x;
  if (c >= chunks) return;
  uint4 a = g[c], b = g[c + rstride16];
  for (int k = 2; k < 10; ++k) {
    const uint4 v = g[c + k * rstride16];
    a.x ^= v.x; a.y ^= v.y; a.z ^= v.z; a.w ^= v.w;
  }
  g[c + 10 * rstride16] = a;
  g[c + 11 * rstride16] = b;
  g[c + 12 * rstride16] = a;
}

int main(int argc, char** argv) {
  const bool spin = argc > 1 && std::string(argv[1]) == "spin";
  if (spin) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  uint8_t* host;
  CK(hipHostMalloc(&host, 13 * 1360));
  memset(host, 1, 13 * 1360);
  uint4* mapped;
  CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&mapped), host, 0));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  struct V { const char* name; int kind; };
  const V vars[] = {{"empty kernel + hipStreamSynchronize", 0},
                    {"empty kernel + event record + hipEventSynchronize", 1},
                    {"mapped (10+3)x1360 touch + hipStreamSynchronize", 2},
                    {"hipStreamSynchronize only (idle stream)", 3},
                    {"empty kernel + hipStreamQuery poll", 4},
                    {"mapped (10+3)x1360 touch + hipStreamQuery poll", 5}};
  for (const V& v : vars) {
    std::vector<double> us;
    for (int i = 0; i < 2200; ++i) {
      const auto t0 = std::chrono::steady_clock::now();
      if (v.kind == 0 || v.kind == 1) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
      if (v.kind == 4) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s);
      if (v.kind == 2 || v.kind == 5) hipLaunchKernelGGL(k_touch, dim3(1), dim3(128), 0, s, mapped, 85, 85);
      if (v.kind >= 4) {
        hipError_t q;
        while ((q = hipStreamQuery(s)) == hipErrorNotReady) {
        }
        CK(q);
      } else if (v.kind == 1) {
        CK(hipEventRecord(ev, s));
        CK(hipEventSynchronize(ev));
      } else {
        CK(hipStreamSynchronize(s));
      }
      const auto t1 = std::chrono::steady_clock::now();
      if (i >= 200) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    std::sort(us.begin(), us.end());
    printf("{\"variant\":\"%s\",\"sched\":\"%s\",\"median_us\":%.2f,\"p10_us\":%.2f,\"p90_us\":%.2f}\n", v.name,
           spin ? "spin" : "default", us[us.size() / 2], us[us.size() / 10], us[us.size() * 9 / 10]);
    fflush(stdout);
  }
  return 0;
}
