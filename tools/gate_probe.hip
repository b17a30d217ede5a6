// gate_probe.hip -- cost of a gated-off launch (the RX dedupe kernels when a
// batch holds no duplicate) against its grid size.  Each variant launches R
// back-to-back kernels that read the gate word and return; per-launch time =
// event span / R.  Not product code.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/gate_probe tools/gate_probe.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

__global__ __launch_bounds__(256) void k_gated(const uint32_t* gate, uint32_t* out) {
  if (*gate == 0u) return;
  out[blockIdx.x * 256 + threadIdx.x] = 1u;
}

// the same with the block-stats LDS prologue of the place kernels
__global__ __launch_bounds__(256) void k_gated_lds(const uint32_t* gate, uint32_t* out) {
  if (*gate == 0u) return;
  __shared__ uint32_t s[5];
  if (threadIdx.x < 5) s[threadIdx.x] = 0;
  __syncthreads();
  out[blockIdx.x * 256 + threadIdx.x] = s[threadIdx.x % 5];
}

int main() {
  uint32_t *gate, *out;
  CK(hipMalloc(&gate, 4));
  CK(hipMalloc(&out, 4096u * 256u * 4u));
  CK(hipMemset(gate, 0, 4));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int R = 200;
  const uint32_t grids[] = {1, 64, 256, 512, 1024, 2048, 4096};
  for (int v = 0; v < 2; ++v)
    for (uint32_t g : grids) {
      float best = 1e30f;
      for (int t = 0; t < 5; ++t) {
        CK(hipEventRecord(e0, s));
        for (int r = 0; r < R; ++r) {
          if (v == 0) k_gated<<<g, 256, 0, s>>>(gate, out);
          else k_gated_lds<<<g, 256, 0, s>>>(gate, out);
        }
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
      }
      printf("{\"variant\":\"%s\",\"blocks\":%u,\"us_per_launch\":%.2f}\n", v ? "gated+lds" : "gated", g,
             best * 1e3f / R);
    }
  return 0;
}
