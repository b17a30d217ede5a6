// txpmc.hip -- TX assembly traffic attribution: the
// production kernel k_tx_c<10,3> and its attribution forms (ATTR in
// ugo_amd/csrc/tx_kernels.hip: 1 = no wire_lens / status stores, 2 = the
// compute-free twin: XOR instead of the network, 3 = both), each launched
// `reps` times over 3 rotated cold input / output sets, one variant after the
// other, so rocprofv3 --pmc passes attribute per kernel name.  argv: reps,
// slot (1488: ugo's packets in 16-B slots; 1536: 128-B aligned slots).
// Timing per variant (hipEvents, median) on stdout as JSON.  Not product code.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/txpmc tools/txpmc.hip
#include "../ugo_amd/csrc/tx_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <random>
#include <string>
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

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  const uint32_t slot = argc > 2 ? static_cast<uint32_t>(atoi(argv[2])) : 1488;
  const uint32_t d = 10, p = 3, n = 13, max_len = 1476, chunks = 93;
  const uint64_t G = 65536;
  if (slot % 16 || slot < 1488) return 2;
  std::mt19937_64 rng(7);
  std::vector<uint8_t> pad(slot);
  for (auto& b : pad) b = static_cast<uint8_t>(rng());
  uint8_t* d_pad;
  CK(hipMalloc(&d_pad, slot));
  CK(hipMemcpy(d_pad, pad.data(), slot, hipMemcpyHostToDevice));
  TxArgs base{};
  base.pad = d_pad;
  base.slot_in = slot;
  base.slot_out = slot;
  base.first_seq = 13 * 1000;
  base.paws = static_cast<uint32_t>((0xffffffffull / n - 1) * n);
  base.max_len = max_len;
  base.chunks = chunks;
  base.d = d;
  base.p = p;
  base.groups = G;
  std::vector<TxArgs> rot(3, base);
  std::vector<uint16_t> L(G * d, static_cast<uint16_t>(max_len));
  for (int r = 0; r < 3; ++r) {
    uint8_t *dp, *w;
    uint16_t *dl, *wl;
    int8_t* st;
    CK(hipMalloc(&dp, G * d * slot));
    CK(hipMalloc(&dl, G * d * 2));
    CK(hipMalloc(&w, G * n * slot));
    CK(hipMalloc(&wl, G * n * 2));
    CK(hipMalloc(&st, G));
    CK(hipMemset(dp, 0x11 * (r + 1), G * d * slot));
    CK(hipMemcpy(dl, L.data(), G * d * 2, hipMemcpyHostToDevice));
    rot[r].pkts = dp;
    rot[r].lens = dl;
    rot[r].wire = w;
    rot[r].wire_lens = wl;
    rot[r].status = st;
  }
  const uint32_t grid = static_cast<uint32_t>((G * chunks + 255) / 256);
  const uint32_t cap = tx_lds_cap();
  struct V {
    std::string name;
    std::function<void(const TxArgs&)> go;
  };
  std::vector<V> vs = {
      {"production k_tx_c<10,3> (ATTR 0)",
       [&](const TxArgs& a) { k_tx_c<10, 3, kTxNT, true, true, 0><<<grid, 256, cap>>>(a); }},
      {"no wire_lens / status stores (ATTR 1)",
       [&](const TxArgs& a) { k_tx_c<10, 3, kTxNT, true, true, 1><<<grid, 256, cap>>>(a); }},
      {"compute-free twin (ATTR 2)",
       [&](const TxArgs& a) { k_tx_c<10, 3, kTxNT, true, true, 2><<<grid, 256, cap>>>(a); }},
      {"compute-free twin, no wire_lens / status stores (ATTR 3)",
       [&](const TxArgs& a) { k_tx_c<10, 3, kTxNT, true, true, 3><<<grid, 256, cap>>>(a); }},
  };
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double alg = double(G) * (d + n) * max_len;
  for (auto& v : vs) {
    std::vector<float> t;
    for (int r = 0; r < reps + 3; ++r) {
      CK(hipEventRecord(e0));
      v.go(rot[r % 3]);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 3) t.push_back(ms * 1000.f);
    }
    std::sort(t.begin(), t.end());
    printf("{\"variant\":\"%s\",\"slot\":%u,\"median_us\":%.2f,\"frac\":%.4f}\n", v.name.c_str(), slot,
           t[t.size() / 2], alg / (t[t.size() / 2] * 1e-6) / 8e12);
  }
  CK(hipGetLastError());
  return 0;
}
