// txpmc.hip -- TX assembly traffic attribution: the
// production kernel k_tx_c<10,3> and its attribution forms (ATTR in
// ugo_amd/csrc/tx_kernels.hip: 1 = no wire_lens / status stores, 2 = the
// compute-free twin: XOR instead of the network, 3 = both), each launched
// `reps` times over 3 rotated cold input / output sets, one variant after the
// other in interleaved rounds (a cache-evicting sweep before each sample),
// rocprofv3 --pmc passes attribute per kernel name.  argv: rounds,
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

// wire_lens and status of a TX batch in a pass of their own: one thread per
// wire packet, consecutive threads on consecutive lengths, so a wave writes
// whole 64-B lines of the length array.  (A/B: k_tx_c ATTR 1 + this kernel
// against k_tx_c, whose chunk-0 lanes store each group's 13 lengths and its
// status one by one.)  Results as tx_data / tx_parity_out:
// bad group -> status ERR_SHARD_SIZE, every length 0; header-only group ->
// ERR_SHARD_NO_DATA, data lengths kept, parity lengths 0; else 0, data lengths,
// parity lengths = the group's longest data packet.
__global__ __launch_bounds__(256) void k_tx_lens(TxArgs a) {
  const uint32_t n = a.d + a.p;
  const uint64_t t = blockIdx.x * 256ull + threadIdx.x;
  if (t >= a.groups * n) return;
  const uint64_t gl = t / n;
  const uint32_t r = static_cast<uint32_t>(t - gl * n);
  const uint64_t g = a.g0 + gl;
  const uint16_t* L = a.lens + g * a.d;
  bool bad = false;
  uint32_t maxsz = 0, mine = 0;
  for (uint32_t k = 0; k < a.d; ++k) {
    const uint32_t Lk = L[k];
    bad |= Lk < kFecHeader || Lk > a.max_len;
    maxsz = max(maxsz, Lk);
    if (k == r) mine = Lk;
  }
  const bool nodata = maxsz <= kFecHeader;
  a.wire_lens[g * n + r] = static_cast<uint16_t>(bad ? 0u : (r < a.d ? mine : (nodata ? 0u : maxsz)));
  if (r == 0 && a.status) a.status[g] = bad ? kBadLength : (nodata ? kNoData : 0);
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

__global__ __launch_bounds__(256) void k_flush(const u32x4* a, uint32_t* out, uint64_t n16) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i >= n16) return;
  const u32x4 v = a[i];
  if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9e3779b9u) out[0] = v.x;
}

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
      {"production k_tx_c<10,3> (ATTR 0; round 5: plain data loads)",
       [&](const TxArgs& a) { k_tx_c<10, 3, kTxNT, true, true, 0><<<grid, 256, cap>>>(a); }},
      {"no wire_lens / status stores (ATTR 1)",
       [&](const TxArgs& a) { k_tx_c<10, 3, kTxNT, true, true, 1><<<grid, 256, cap>>>(a); }},
      {"compute-free twin (ATTR 2)",
       [&](const TxArgs& a) { k_tx_c<10, 3, kTxNT, true, true, 2><<<grid, 256, cap>>>(a); }},
      {"compute-free twin, no wire_lens / status stores (ATTR 3)",
       [&](const TxArgs& a) { k_tx_c<10, 3, kTxNT, true, true, 3><<<grid, 256, cap>>>(a); }},
      {"XCD-contiguous blocks (ATTR 4)",
       [&](const TxArgs& a) { k_tx_c<10, 3, kTxNT, true, true, 4><<<grid, 256, cap>>>(a); }},
      {"resident grid: 512 blocks (2 per CU) striding, no residency LDS (ATTR 64)",
       [&](const TxArgs& a) { k_tx_c<10, 3, kTxNT, true, true, 64><<<512, 256, 16u * a.chunks>>>(a); }},
      {"resident grid: 768 blocks (3 per CU) striding, no residency LDS (ATTR 64)",
       [&](const TxArgs& a) { k_tx_c<10, 3, kTxNT, true, true, 64><<<768, 256, 16u * a.chunks>>>(a); }},
      {"runs of 4 blocks per XCD (ATTR 16)",
       [&](const TxArgs& a) { k_tx_c<10, 3, kTxNT, true, true, 16><<<grid, 256, cap>>>(a); }},
      {"runs of 8 blocks per XCD (ATTR 32)",
       [&](const TxArgs& a) { k_tx_c<10, 3, kTxNT, true, true, 32><<<grid, 256, cap>>>(a); }},
      {"nontemporal data loads, the round-4 production (ATTR 8)",
       [&](const TxArgs& a) { k_tx_c<10, 3, kTxNT, true, true, 8><<<grid, 256, cap>>>(a); }},
      {"XCD-contiguous blocks, nontemporal data loads (ATTR 12)",
       [&](const TxArgs& a) { k_tx_c<10, 3, kTxNT, true, true, 12><<<grid, 256, cap>>>(a); }},
      {"no wire_lens / status stores + k_tx_lens (ATTR 1 + lens kernel)", [&](const TxArgs& a) {
         k_tx_c<10, 3, kTxNT, true, true, 1><<<grid, 256, cap>>>(a);
         k_tx_lens<<<static_cast<uint32_t>((a.groups * 13 + 255) / 256), 256>>>(a);
       }},
  };
  {  // ATTR 1 + k_tx_lens writes the same wire, wire_lens and status as production (random lengths)
    std::vector<uint16_t> Lr(G * d);
    for (auto& v : Lr) v = static_cast<uint16_t>(6 + rng() % (max_len - 5));
    for (uint64_t g = 0; g < G; g += 97) Lr[g * d + 3] = 5;  // bad
    for (uint64_t g = 1; g < G; g += 89)
      for (uint32_t k = 0; k < d; ++k) Lr[g * d + k] = 6;  // header-only
    TxArgs x = rot[0], y = rot[1];
    uint16_t* dl;
    CK(hipMalloc(&dl, G * d * 2));
    CK(hipMemcpy(dl, Lr.data(), G * d * 2, hipMemcpyHostToDevice));
    x.lens = y.lens = dl;
    y.pkts = x.pkts;
    for (const TxArgs* t : {&x, &y}) {
      CK(hipMemset(t->wire, 0x5c, G * n * slot));
      CK(hipMemset(t->wire_lens, 0x77, G * n * 2));
      CK(hipMemset(t->status, 0x33, G));
    }
    k_tx_c<10, 3, kTxNT, true, true, 0><<<grid, 256, cap>>>(x);
    k_tx_c<10, 3, kTxNT, true, true, 1><<<grid, 256, cap>>>(y);
    k_tx_lens<<<static_cast<uint32_t>((G * 13 + 255) / 256), 256>>>(y);
    CK(hipDeviceSynchronize());
    std::vector<uint8_t> w1(G * n * slot), w2(G * n * slot);
    std::vector<uint16_t> l1(G * n), l2(G * n);
    std::vector<int8_t> s1(G), s2(G);
    CK(hipMemcpy(w1.data(), x.wire, w1.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(w2.data(), y.wire, w2.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(l1.data(), x.wire_lens, G * n * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(l2.data(), y.wire_lens, G * n * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(s1.data(), x.status, G, hipMemcpyDeviceToHost));
    CK(hipMemcpy(s2.data(), y.status, G, hipMemcpyDeviceToHost));
    printf("{\"check\":\"ATTR 1 + k_tx_lens == production (wire, wire_lens, status)\",\"same\":%s}\n",
           (w1 == w2 && l1 == l2 && s1 == s2) ? "true" : "false");
    // the resident striding grid (ATTR 64) against production
    CK(hipMemset(y.wire, 0x5c, G * n * slot));
    CK(hipMemset(y.wire_lens, 0x77, G * n * 2));
    CK(hipMemset(y.status, 0x33, G));
    k_tx_c<10, 3, kTxNT, true, true, 64><<<512, 256, 16u * y.chunks>>>(y);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(w2.data(), y.wire, w2.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(l2.data(), y.wire_lens, G * n * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(s2.data(), y.status, G, hipMemcpyDeviceToHost));
    printf("{\"check\":\"resident 512-block grid (ATTR 64) == production (wire, wire_lens, status)\",\"same\":%s}\n",
           (w1 == w2 && l1 == l2 && s1 == s2) ? "true" : "false");
    CK(hipFree(dl));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double alg = double(G) * (d + n) * max_len;
  // interleaved rounds: every variant once per round, each sample after a
  // cache-evicting sweep, 3 launches on the 3 rotated sets; medians
  const uint64_t fl16 = (768ull << 20) / 16;
  uint8_t* fl = nullptr;
  CK(hipMalloc(&fl, fl16 * 16));
  CK(hipMemset(fl, 1, fl16 * 16));
  std::vector<std::vector<float>> t(vs.size());
  for (int w = 0; w < 2; ++w)
    for (auto& v : vs) v.go(rot[w % 3]);
  CK(hipDeviceSynchronize());
  for (int r = 0; r < reps; ++r)
    for (size_t k = 0; k < vs.size(); ++k) {
      k_flush<<<static_cast<uint32_t>((fl16 + 255) / 256), 256>>>(reinterpret_cast<const u32x4*>(fl),
                                                                  reinterpret_cast<uint32_t*>(fl), fl16);
      CK(hipEventRecord(e0));
      for (int j = 0; j < 3; ++j) vs[k].go(rot[j]);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[k].push_back(ms * 1000.f / 3.f);
    }
  for (size_t k = 0; k < vs.size(); ++k) {
    std::sort(t[k].begin(), t[k].end());
    const double med = t[k][t[k].size() / 2];
    printf("{\"variant\":\"%s\",\"slot\":%u,\"median_us\":%.2f,\"min_us\":%.2f,\"frac\":%.4f}\n",
           vs[k].name.c_str(), slot, med, t[k][0], alg / (med * 1e-6) / 8e12);
  }
  CK(hipGetLastError());
  return 0;
}
