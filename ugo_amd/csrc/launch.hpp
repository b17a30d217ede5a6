// launch.hpp -- every kernel launch of the engine goes through ugo::kern::launch().
//
// Normally that is a plain hipLaunchKernelGGL.  While a context has launch
// timing on (ugo_fec_timing_begin, include/ugo_fec.h), the launch is issued
// with hipExtLaunchKernel start/stop events instead: the events then carry the
// dispatch's own begin/end timestamps (the clock rocprofv3's kernel trace
// reads), so a bench gets per-kernel durations without event-record packets --
// and their cache-release fences -- between the kernels it times.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace ugo {
namespace kern {

// kernel classes reported by ugo_fec_timing_end (UGO_FEC_KERNEL_* in ugo_fec.h)
enum KernelId : uint32_t {
  kKEncode = 1,       // encode (compile-time network or descriptor form)
  kKReconstruct = 2,  // reconstruct (descriptor apply)
  kKPrepare = 3,      // per-group decode descriptors (d + p > 16)
  kKBytes = 4,        // byte-granular encode / reconstruct (unaligned layouts)
  kKRx = 5,           // RX group assembly
  kKTx = 6,           // TX group assembly
  kKPacket = 7,       // packet wire decode
};

struct LaunchTimer {
  hipEvent_t* ev = nullptr;  // 2 * cap events: start, stop of launch i at 2i, 2i+1
  uint32_t* kid = nullptr;   // kernel class of launch i
  size_t cap = 0, used = 0, dropped = 0;
};

// The timer of the context whose ABI call runs on this thread (set for the
// duration of the call by ugo_fec.cpp), or null.
LaunchTimer*& current_timer();

template <typename F, typename... Args>
inline void launch(uint32_t kid, F kernel, const dim3& grid, const dim3& block, uint32_t shmem, hipStream_t s,
                   Args... args) {
  LaunchTimer* t = current_timer();
  if (t != nullptr) {
    if (t->used < t->cap) {
      const size_t i = t->used++;
      t->kid[i] = kid;
      hipExtLaunchKernelGGL(kernel, grid, block, shmem, s, t->ev[2 * i], t->ev[2 * i + 1], 0u, args...);
      return;
    }
    ++t->dropped;
  }
  hipLaunchKernelGGL(kernel, grid, block, shmem, s, args...);
}

}  // namespace kern
}  // namespace ugo
