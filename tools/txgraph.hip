// txgraph.hip -- the host TX pipeline of ugo_fec_tx_assemble_host (data
// packets H2D on one stream, k_tx_c on another, wire packets D2H on a third,
// joined by events through 4 device stages) enqueued directly, as the library
// does, against the same work captured once into a HIP graph and launched:
// does a graph keep many small chunks from slowing down (past ~40 chunks per
// call the direct form ran 2-4x slower, profiles/r5/host_tx_chunk_ab*)?
// 65,536 (10+3) groups of 1476-B packets, 1488-B slots, pinned buffers; chunk
// sizes from argv (MiB of input + output per chunk).  Median wall ms per call
// as JSON.  Not product code.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/txgraph tools/txgraph.hip
#include "../ugo_amd/csrc/tx_kernels.hip"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

namespace ugo {
namespace kern {
LaunchTimer*& current_timer() {
  static thread_local LaunchTimer* t = nullptr;
  return t;
}
}  // namespace kern
}  // namespace ugo

using namespace ugo::kern;

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

constexpr int kStages = 4;

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 7;
  const uint64_t G = argc > 2 ? strtoull(argv[2], nullptr, 10) : 65536;
  const uint32_t d = 10, p = 3, n = 13, max_len = 1476, slot = 1488, chunks = 93;
  const uint64_t per_group = uint64_t(d + n) * slot;
  uint8_t *pk, *wire;
  uint16_t *lens, *wl;
  CK(hipHostMalloc(&pk, G * d * slot));
  CK(hipHostMalloc(&wire, G * n * slot));
  CK(hipHostMalloc(&lens, G * d * 2));
  CK(hipHostMalloc(&wl, G * n * 2));
  std::mt19937_64 rng(3);
  for (uint64_t i = 0; i < G * d * slot / 8; ++i) reinterpret_cast<uint64_t*>(pk)[i] = rng();
  for (uint64_t i = 0; i < G * d; ++i) lens[i] = max_len;
  // argv[3]: streams created (and used once for a small copy each) before the pipeline's three,
  // to see whether the copy engines a stream gets depend on creation order
  const int dummies = argc > 3 ? atoi(argv[3]) : 0;
  std::vector<hipStream_t> dummy(dummies);
  uint8_t* dtmp;
  CK(hipMalloc(&dtmp, 4096));
  for (auto& x : dummy) {
    CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    CK(hipMemcpyAsync(dtmp, pk, 4096, hipMemcpyHostToDevice, x));
    CK(hipStreamSynchronize(x));
  }
  hipStream_t sk, sin, sout;
  CK(hipStreamCreateWithFlags(&sk, hipStreamNonBlocking));
  {  // as the library: the H2D stream from the low-priority class (a hardware queue apart)
    int least = 0, greatest = 0;
    CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    CK(hipStreamCreateWithPriority(&sin, hipStreamNonBlocking, least));
  }
  CK(hipStreamCreateWithFlags(&sout, hipStreamNonBlocking));
  uint8_t* dpad;
  CK(hipMalloc(&dpad, slot));
  CK(hipMemset(dpad, 0x5a, slot));
  uint16_t *dlens, *dwl;
  CK(hipMalloc(&dlens, G * d * 2));
  CK(hipMalloc(&dwl, G * n * 2));
  const uint64_t max_stage = 64ull << 20;
  uint8_t* stages;
  CK(hipMalloc(&stages, kStages * (max_stage + 4096)));
  hipEvent_t ev[3 * kStages + 2];
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  TxArgs a{};
  a.slot_in = slot;
  a.slot_out = slot;
  a.paws = static_cast<uint32_t>((0xffffffffull / n - 1) * n);
  a.max_len = max_len;
  a.chunks = chunks;
  a.d = d;
  a.p = p;
  a.pad = dpad;
  // the pipeline of ugo_fec_tx_assemble_host, every call on sk / sin / sout
  auto enqueue = [&](uint64_t cg) {
    const uint64_t o_wire = (cg * d * slot + 255) / 256 * 256, sbytes = o_wire + (cg * n * slot + 255) / 256 * 256;
    CK(hipEventRecord(ev[3 * kStages], sk));
    CK(hipStreamWaitEvent(sin, ev[3 * kStages], 0));
    CK(hipStreamWaitEvent(sout, ev[3 * kStages], 0));
    CK(hipMemcpyAsync(dlens, lens, G * d * 2, hipMemcpyHostToDevice, sin));
    uint64_t k = 0;
    for (uint64_t g0 = 0; g0 < G; g0 += cg, ++k) {
      const uint64_t gn = std::min(cg, G - g0);
      const int b = static_cast<int>(k % kStages);
      uint8_t* sb = stages + b * sbytes;
      if (k >= kStages) CK(hipStreamWaitEvent(sin, ev[2 * kStages + b], 0));
      CK(hipMemcpyAsync(sb, pk + g0 * d * slot, gn * d * slot, hipMemcpyHostToDevice, sin));
      CK(hipEventRecord(ev[b], sin));
      CK(hipStreamWaitEvent(sk, ev[b], 0));
      a.pkts = sb;
      a.lens = dlens + g0 * d;
      a.wire = sb + o_wire;
      a.wire_lens = dwl + g0 * n;
      a.status = nullptr;
      a.first_seq = static_cast<uint32_t>((g0 * n) % a.paws);
      a.g0 = 0;
      a.groups = gn;
      CK(launch_tx_assemble(0, a, sk));
      CK(hipEventRecord(ev[kStages + b], sk));
      CK(hipStreamWaitEvent(sout, ev[kStages + b], 0));
      CK(hipMemcpyAsync(wire + g0 * n * slot, sb + o_wire, gn * n * slot, hipMemcpyDeviceToHost, sout));
      CK(hipEventRecord(ev[2 * kStages + b], sout));
    }
    CK(hipMemcpyAsync(wl, dwl, G * n * 2, hipMemcpyDeviceToHost, sout));
    // join onto sk (a capture must end on its origin stream)
    CK(hipEventRecord(ev[3 * kStages + 1], sin));
    CK(hipStreamWaitEvent(sk, ev[3 * kStages + 1], 0));
    CK(hipEventRecord(ev[3 * kStages + 1], sout));
    CK(hipStreamWaitEvent(sk, ev[3 * kStages + 1], 0));
  };
  auto med = [](std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  std::vector<uint8_t> ref;
  for (int mib : {64, 16}) {
    const uint64_t cg = std::max<uint64_t>(1, std::min<uint64_t>((G + 7) / 8, (uint64_t(mib) << 20) / per_group));
    const uint64_t nch = (G + cg - 1) / cg;
    // direct
    std::vector<double> td, te;
    for (int r = 0; r <= reps; ++r) {
      const auto t0 = std::chrono::steady_clock::now();
      enqueue(cg);
      const auto t1 = std::chrono::steady_clock::now();
      CK(hipStreamSynchronize(sk));
      if (r) {
        td.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        te.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
      }
    }
    if (ref.empty()) ref.assign(wire, wire + G * n * slot);
    const bool same_direct = std::equal(ref.begin(), ref.end(), wire);
    // graph: captured once, launched reps times
    const auto c0 = std::chrono::steady_clock::now();
    hipGraph_t graph;
    hipGraphExec_t exec;
    CK(hipStreamBeginCapture(sk, hipStreamCaptureModeThreadLocal));
    enqueue(cg);
    CK(hipStreamEndCapture(sk, &graph));
    CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    const double build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - c0).count();
    std::memset(wire, 0, G * n * slot);
    std::vector<double> tg;
    for (int r = 0; r <= reps; ++r) {
      const auto t0 = std::chrono::steady_clock::now();
      CK(hipGraphLaunch(exec, sk));
      CK(hipStreamSynchronize(sk));
      if (r) tg.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    const bool same_graph = std::equal(ref.begin(), ref.end(), wire);
    CK(hipGraphExecDestroy(exec));
    CK(hipGraphDestroy(graph));
    printf("{\"dummy_streams\":%d,\"chunk_mib\":%d,\"groups\":%llu,\"chunks\":%llu,\"direct_ms\":%.3f,\"direct_enqueue_ms\":%.3f,"
           "\"graph_ms\":%.3f,\"graph_build_ms\":%.3f,\"same_direct\":%s,\"same_graph\":%s}\n",
           dummies, mib, (unsigned long long)G, (unsigned long long)nch, med(td), med(te), med(tg), build_ms,
           same_direct ? "true" : "false", same_graph ? "true" : "false");
    fflush(stdout);
  }
  return 0;
}
