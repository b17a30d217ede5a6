// membench.hip -- HBM ceilings on MI355X for the FEC access pattern.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/membench tools/membench.hip
// Prints one JSON object per variant: GB/s over the bytes each variant moves.
//   copy16      : float4 copy, N bytes read + N bytes written (the guide's 6.29 TB/s figure)
//   read16      : read-only stream (xor-reduce), N bytes
//   pattern     : the (10+3)x1360 encode layout with XOR instead of GF math:
//                 10 rows read, 3 rows written per group (no compute ceiling)
//   pattern_nt  : same with nontemporal loads/stores
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__global__ void k_copy(const uint4* __restrict__ a, uint4* __restrict__ b, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) b[i] = a[i];
}

__global__ void k_read(const uint4* __restrict__ a, uint4* __restrict__ out, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (; i < n; i += stride) {
    uint4 v = a[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = make_uint4(acc, 0, 0, 0);
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// copy with U independent loads in flight per thread before the stores
template <int U, bool NTS>
__global__ __launch_bounds__(256) void k_copyu(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
  size_t i = (blockIdx.x * (size_t)blockDim.x + threadIdx.x);
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = a[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NTS) __builtin_nontemporal_store(v[u], &b[i + u * stride]);
      else b[i + u * stride] = v[u];
    }
  }
}

__global__ __launch_bounds__(256) void k_write(u32x4* __restrict__ b, size_t n) {
  size_t i = (blockIdx.x * (size_t)blockDim.x + threadIdx.x);
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  u32x4 v = {1u, 2u, 3u, (uint32_t)i};
  for (; i < n; i += stride) b[i] = v;
}

template <bool NT>
__global__ __launch_bounds__(256) void k_pattern(uint8_t* base, uint32_t items, uint32_t chunks, uint64_t pitch,
                                                 uint64_t group_bytes) {
  uint32_t item = blockIdx.x * 256u + threadIdx.x;
  if (item >= items) return;
  uint32_t g = item / chunks, c = item - g * chunks;
  uint8_t* gp = base + g * group_bytes + c * 16ull;
  uint4 x[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) {
    const u32x4* p = reinterpret_cast<const u32x4*>(gp + (uint64_t)k * pitch);
    u32x4 v = NT ? __builtin_nontemporal_load(p) : *p;
    x[k] = make_uint4(v.x, v.y, v.z, v.w);
  }
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    uint4 y = x[i];
#pragma unroll
    for (int k = 3; k < 10; ++k) {
      if ((k + i) & 1) {
        y.x ^= x[k].x; y.y ^= x[k].y; y.z ^= x[k].z; y.w ^= x[k].w;
      }
    }
    u32x4* q = reinterpret_cast<u32x4*>(gp + (uint64_t)(10 + i) * pitch);
    u32x4 v = {y.x, y.y, y.z, y.w};
    if (NT) {
      __builtin_nontemporal_store(v, q);
    } else {
      *q = v;
    }
  }
}

#define GPTR(p) ((const __attribute__((address_space(1))) void*)(p))
#define LPTR(p) ((__attribute__((address_space(3))) void*)(p))

// read-only, one 16-B chunk per thread over a full grid, NT loads (encode's load form)
__global__ __launch_bounds__(256) void k_read_full(const u32x4* __restrict__ a, uint32_t* out, size_t n) {
  const size_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i >= n) return;
  const u32x4 v = __builtin_nontemporal_load(&a[i]);
  if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345678u) out[0] = 1u;
}

// read-only through LDS-DMA (global_load_lds_dwordx4): U 1-KiB pieces per wave
// in flight, wave-private LDS, grid-stride; AUX 2 = nt
template <int U, int AUX>
__global__ __launch_bounds__(256) void k_read_glds(const uint8_t* a, uint32_t* out, size_t n16) {
  __shared__ u32x4 buf[4][U][64];
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const size_t nw = gridDim.x * 4ull;
  uint32_t acc = 0;
  for (size_t base = (blockIdx.x * 4ull + w) * 64u * U; base < n16; base += nw * 64u * U) {
#pragma unroll
    for (int u = 0; u < U; ++u)
      __builtin_amdgcn_global_load_lds(GPTR(a + (base + u * 64u + lane) * 16u), LPTR(&buf[w][u][0]), 16, 0, AUX);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    acc ^= buf[w][lane & (U - 1)][lane].x;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// the planar encode pattern with the 10 row loads through LDS-DMA
template <int AUX>
__global__ __launch_bounds__(256) void k_pattern_glds(uint8_t* base, uint32_t items, uint32_t chunks, uint64_t pitch,
                                                      uint64_t group_bytes) {
  __shared__ u32x4 buf[4][10][64];
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  uint32_t item = blockIdx.x * 256u + threadIdx.x;
  if (item >= items) return;
  uint32_t g = item / chunks, c = item - g * chunks;
  uint8_t* gp = base + g * group_bytes + c * 16ull;
#pragma unroll
  for (int k = 0; k < 10; ++k) __builtin_amdgcn_global_load_lds(GPTR(gp + (uint64_t)k * pitch), LPTR(&buf[w][k][0]), 16, 0, AUX);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  u32x4 x[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) x[k] = buf[w][k][lane];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    u32x4 y = x[i];
#pragma unroll
    for (int k = 3; k < 10; ++k)
      if ((k + i) & 1) y ^= x[k];
    *reinterpret_cast<u32x4*>(gp + (uint64_t)(10 + i) * pitch) = y;
  }
}

int main(int argc, char** argv) {
  const size_t G = 65536, n = 13, pitch = 1360, S = 1350;
  const size_t bytes = G * n * pitch;
  uint8_t *a, *b;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 1, bytes));
  CK(hipMemset(b, 2, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 20;
  auto timeit = [&](auto launch) -> float {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
  };
  const size_t n16 = bytes / 16;
  for (int grid : {2048, 4096, 8192}) {
    float ms = timeit([&] { hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, n16); return 0; });
    printf("{\"variant\":\"copy16\",\"grid\":%d,\"bytes\":%zu,\"us\":%.2f,\"GBps\":%.1f}\n", grid, 2 * bytes, ms * 1e3,
           2.0 * bytes / (ms * 1e-3) / 1e9);
    ms = timeit([&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, n16); return 0; });
    printf("{\"variant\":\"read16\",\"grid\":%d,\"bytes\":%zu,\"us\":%.2f,\"GBps\":%.1f}\n", grid, bytes, ms * 1e3,
           1.0 * bytes / (ms * 1e-3) / 1e9);
  }
  for (int grid : {4096, 16384}) {
    float ms = timeit([&] { hipLaunchKernelGGL((k_copyu<4, false>), dim3(grid), dim3(256), 0, 0, (const u32x4*)a, (u32x4*)b, n16); return 0; });
    printf("{\"variant\":\"copy_u4\",\"grid\":%d,\"GBps\":%.1f}\n", grid, 2.0 * bytes / (ms * 1e-3) / 1e9);
    ms = timeit([&] { hipLaunchKernelGGL((k_copyu<4, true>), dim3(grid), dim3(256), 0, 0, (const u32x4*)a, (u32x4*)b, n16); return 0; });
    printf("{\"variant\":\"copy_u4_nts\",\"grid\":%d,\"GBps\":%.1f}\n", grid, 2.0 * bytes / (ms * 1e-3) / 1e9);
    ms = timeit([&] { hipLaunchKernelGGL((k_copyu<8, false>), dim3(grid), dim3(256), 0, 0, (const u32x4*)a, (u32x4*)b, n16); return 0; });
    printf("{\"variant\":\"copy_u8\",\"grid\":%d,\"GBps\":%.1f}\n", grid, 2.0 * bytes / (ms * 1e-3) / 1e9);
    ms = timeit([&] { hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, (u32x4*)b, n16); return 0; });
    printf("{\"variant\":\"write16\",\"grid\":%d,\"GBps\":%.1f}\n", grid, 1.0 * bytes / (ms * 1e-3) / 1e9);
  }
  const uint32_t chunks = 85, items = G * chunks;
  const double alg = (double)G * n * S;
  const double moved = (double)G * n * pitch;
  for (int planar = 0; planar < 2; ++planar) {
    // interleaved [G][13][pitch] vs planar [13][G][pitch] (row stride G*pitch, group stride pitch)
    const uint64_t rs = planar ? G * pitch : pitch, gs = planar ? pitch : n * pitch;
    float ms = timeit([&] { hipLaunchKernelGGL(k_pattern<false>, dim3((items + 255) / 256), dim3(256), 0, 0, a, items, chunks, rs, gs); return 0; });
    printf("{\"variant\":\"pattern%s\",\"us\":%.2f,\"alg_GBps\":%.1f,\"moved_GBps\":%.1f}\n", planar ? "_planar" : "", ms * 1e3,
           alg / (ms * 1e-3) / 1e9, moved / (ms * 1e-3) / 1e9);
    ms = timeit([&] { hipLaunchKernelGGL(k_pattern<true>, dim3((items + 255) / 256), dim3(256), 0, 0, a, items, chunks, rs, gs); return 0; });
    printf("{\"variant\":\"pattern_nt%s\",\"us\":%.2f,\"alg_GBps\":%.1f,\"moved_GBps\":%.1f}\n", planar ? "_planar" : "", ms * 1e3,
           alg / (ms * 1e-3) / 1e9, moved / (ms * 1e-3) / 1e9);
  }
  for (int aux : {0, 2}) {
    const uint64_t rs = G * pitch, gs = pitch;
    float ms = timeit([&] {
      if (aux) hipLaunchKernelGGL(k_pattern_glds<2>, dim3((items + 255) / 256), dim3(256), 0, 0, a, items, chunks, rs, gs);
      else hipLaunchKernelGGL(k_pattern_glds<0>, dim3((items + 255) / 256), dim3(256), 0, 0, a, items, chunks, rs, gs);
      return 0; });
    printf("{\"variant\":\"pattern_glds_planar aux%d\",\"us\":%.2f,\"alg_GBps\":%.1f,\"moved_GBps\":%.1f}\n", aux, ms * 1e3,
           alg / (ms * 1e-3) / 1e9, moved / (ms * 1e-3) / 1e9);
  }
  {
    float ms = timeit([&] { hipLaunchKernelGGL(k_read_full, dim3((n16 + 255) / 256), dim3(256), 0, 0, (const u32x4*)a, (uint32_t*)b, n16); return 0; });
    printf("{\"variant\":\"read16 full-grid nt\",\"GBps\":%.1f}\n", bytes / (ms * 1e-3) / 1e9);
    const size_t n16r = n16 / 1024 * 1024;
    for (int grid : {1024, 2048, 4096}) {
      ms = timeit([&] { hipLaunchKernelGGL((k_read_glds<4, 2>), dim3(grid), dim3(256), 0, 0, (const uint8_t*)a, (uint32_t*)b, n16r); return 0; });
      printf("{\"variant\":\"read glds U4 nt\",\"grid\":%d,\"GBps\":%.1f}\n", grid, n16r * 16.0 / (ms * 1e-3) / 1e9);
      ms = timeit([&] { hipLaunchKernelGGL((k_read_glds<8, 2>), dim3(grid), dim3(256), 0, 0, (const uint8_t*)a, (uint32_t*)b, n16r); return 0; });
      printf("{\"variant\":\"read glds U8 nt\",\"grid\":%d,\"GBps\":%.1f}\n", grid, n16r * 16.0 / (ms * 1e-3) / 1e9);
      ms = timeit([&] { hipLaunchKernelGGL((k_read_glds<8, 0>), dim3(grid), dim3(256), 0, 0, (const uint8_t*)a, (uint32_t*)b, n16r); return 0; });
      printf("{\"variant\":\"read glds U8 default\",\"grid\":%d,\"GBps\":%.1f}\n", grid, n16r * 16.0 / (ms * 1e-3) / 1e9);
    }
  }
  return 0;
}
