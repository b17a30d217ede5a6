// txgroup.hip -- TX assembly: k_tx_c (one thread per chunk of a group, round 1-3
// production) against k_tx_g (one block per group, streaming), and the nt copy
// of the same bytes, cold regime (3 rotated input / output sets, a cache-
// evicting sweep before every sample), interleaved, medians.  Both kernels are
// first checked byte for byte against each other (wire, wire_lens, status) on
// random lengths (short, header-only and bad groups included).  Not product
// code.  argv: rounds.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/txgroup tools/txgroup.hip
#include "../ugo_amd/csrc/tx_kernels.hip"
#include "tx_experiments.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <random>
#include <string>
#include <vector>

#include "../ugo_amd/csrc/gf256.hpp"

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

__global__ __launch_bounds__(256) void k_copy1(const u32x4* src, u32x4* dst, uint64_t n16) {
  const uint64_t c = blockIdx.x * 256ull + threadIdx.x;
  if (c >= n16) return;
  __builtin_nontemporal_store(__builtin_nontemporal_load(src + c), dst + c);
}

// One thread per 16-B chunk of a WIRE packet (one chunk per thread, full grid,
// the copy's shape): a data chunk is one load and one store; a parity chunk
// loads the 10 data chunks of its column (just read by the group's data
// threads: L2 / Infinity-Cache hits) and folds its own row of the network.
// SWZ 1: XCD-contiguous blocks, so a group's data and parity blocks share an L2.
template <int D, int P, int SWZ, int I>
__device__ __forceinline__ V4 tx_row(const V4* x) {
  return cparity<D, P, I>(x);
}
template <int D, int P, int SWZ>
__global__ __launch_bounds__(256) void k_tx_o(TxArgs a) {
  const uint32_t n = D + P, nch = a.chunks;
  const uint32_t t = block_id<SWZ>() * 256u + threadIdx.x;
  if (t >= a.groups * n * nch) return;
  const uint32_t gl = t / (n * nch), rem = t - gl * n * nch, r = rem / nch, m = rem - r * nch, o = 16u * m;
  const uint64_t g = a.g0 + gl;
  uint32_t Ls[D];
  bool bad = false;
  uint32_t maxsz = 0;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    Ls[k] = a.lens[g * D + k];
    bad |= Ls[k] < 6u || Ls[k] > a.max_len;
    maxsz = max(maxsz, Ls[k]);
  }
  if (bad) {
    if (m == 0) {
      a.wire_lens[g * n + r] = 0;
      if (r == 0 && a.status) a.status[g] = kBadLength;
    }
    return;
  }
  const uint32_t seq0 = static_cast<uint32_t>((uint64_t(a.first_seq) + g * n) % a.paws);
  const uint8_t* src = a.pkts + g * D * a.slot_in + o;
  uint8_t* dst = a.wire + (g * n + r) * a.slot_out + o;
  if (r < static_cast<uint32_t>(D)) {
    const uint32_t Lk = Ls[r];
    if (o < Lk) {
      V4 w = keep_bytes(load16<1>(src + uint64_t(r) * a.slot_in), Lk - o);
      if (m == 0) put_header(w, seq0 + r, kTypeData);
      if (a.pad) xor4(w, load16<0>(a.pad + o));
      store16<kTxNT>(dst, keep_bytes(w, Lk - o), 16u);
    }
    if (m == 0) {
      a.wire_lens[g * n + r] = static_cast<uint16_t>(Lk);
      if (r == 0 && a.status) a.status[g] = maxsz <= kFecHeader ? kNoData : 0;
    }
    return;
  }
  if (maxsz <= kFecHeader) {  // header-only group: no parity
    if (m == 0) a.wire_lens[g * n + r] = 0;
    return;
  }
  if (m == 0) a.wire_lens[g * n + r] = static_cast<uint16_t>(maxsz);
  if (o >= maxsz) return;
  V4 x[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    x[k] = V4{{0u, 0u, 0u, 0u}};
    if (o < Ls[k]) x[k] = keep_bytes(load16<0>(src + uint64_t(k) * a.slot_in), Ls[k] - o);
    if (m == 0) {
      x[k].v[0] = 0u;
      x[k].v[1] &= 0xffff0000u;
    }
  }
  V4 y;
  const uint32_t i = r - D;
  if (i == 0) y = cparity<D, P, 0>(x);
  else if (i == 1) y = cparity<D, P, 1>(x);
  else y = cparity<D, P, 2>(x);
  if (m == 0) put_header(y, seq0 + r, kTypeFEC);
  if (a.pad) xor4(y, load16<0>(a.pad + o));
  store16<kTxNT>(dst, keep_bytes(y, maxsz - o), 16u);
}

__global__ __launch_bounds__(256) void k_flush(const u32x4* a, uint32_t* out, uint64_t n16) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i >= n16) return;
  const u32x4 v = a[i];
  if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9e3779b9u) out[0] = v.x;
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 11;
  const uint32_t d = 10, p = 3, n = 13, max_len = 1476, slot = 1488, chunks = 93;
  std::mt19937_64 rng(7);
  std::vector<uint8_t> pad(slot);
  for (auto& b : pad) b = static_cast<uint8_t>(rng());
  uint8_t* d_pad;
  CK(hipMalloc(&d_pad, slot));
  CK(hipMemcpy(d_pad, pad.data(), slot, hipMemcpyHostToDevice));
  TxArgs base{};
  base.pad = d_pad;
  base.desc = nullptr;
  base.slot_in = slot;
  base.slot_out = slot;
  base.first_seq = 13 * 1000;
  base.paws = static_cast<uint32_t>((0xffffffffull / n - 1) * n);
  base.max_len = max_len;
  base.chunks = chunks;
  base.d = d;
  base.p = p;
  const uint32_t lds = d * chunks * 16;
  auto run_c = [&](TxArgs a) {
    k_tx_c<10, 3, kTxNT, true><<<static_cast<uint32_t>((a.groups * a.chunks + 255) / 256), 256, tx_lds_cap()>>>(a);
  };
  auto run_cl = [&](TxArgs a) {
    k_tx_c<10, 3, kTxNT, true, true><<<static_cast<uint32_t>((a.groups * a.chunks + 255) / 256), 256, tx_lds_cap()>>>(a);
  };
  auto run_cl_cap = [&](TxArgs a, uint32_t lds) {
    k_tx_c<10, 3, kTxNT, true, true><<<static_cast<uint32_t>((a.groups * a.chunks + 255) / 256), 256, lds>>>(a);
  };
  auto run_g = [&](TxArgs a) { k_tx_g<10, 3><<<static_cast<uint32_t>(a.groups), 256, lds>>>(a); };
  auto run_o = [&](TxArgs a, int swz) {
    const uint32_t blocks = static_cast<uint32_t>((a.groups * 13 * a.chunks + 255) / 256);
    if (swz)
      k_tx_o<10, 3, 1><<<blocks, 256>>>(a);
    else
      k_tx_o<10, 3, 0><<<blocks, 256>>>(a);
  };

  // ---- check: random lengths incl. short, header-only groups and bad groups
  {
    const uint64_t G = 4096;
    std::vector<uint8_t> pk(G * d * slot);
    for (auto& b : pk) b = static_cast<uint8_t>(rng());
    std::vector<uint16_t> L(G * d);
    for (uint64_t g = 0; g < G; ++g)
      for (uint32_t k = 0; k < d; ++k) {
        uint16_t v = static_cast<uint16_t>(6 + rng() % (max_len - 5));
        if (g % 97 == 3) v = 6;                          // header-only group
        if (g % 131 == 5 && k == 2) v = 5;               // bad length
        if (g % 7 == 0) v = max_len;                     // full
        L[g * d + k] = v;
      }
    uint8_t *dp, *w1, *w2;
    uint16_t *dl, *l1, *l2;
    int8_t *s1, *s2;
    CK(hipMalloc(&dp, pk.size()));
    CK(hipMalloc(&dl, L.size() * 2));
    CK(hipMalloc(&w1, G * n * slot));
    CK(hipMalloc(&w2, G * n * slot));
    CK(hipMalloc(&l1, G * n * 2));
    CK(hipMalloc(&l2, G * n * 2));
    CK(hipMalloc(&s1, G));
    CK(hipMalloc(&s2, G));
    CK(hipMemcpy(dp, pk.data(), pk.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dl, L.data(), L.size() * 2, hipMemcpyHostToDevice));
    for (uint8_t* w : {w1, w2}) CK(hipMemset(w, 0x5c, G * n * slot));
    for (uint16_t* l : {l1, l2}) CK(hipMemset(l, 0x77, G * n * 2));
    for (int8_t* st : {s1, s2}) CK(hipMemset(st, 0x33, G));
    TxArgs a = base;
    a.pkts = dp;
    a.lens = dl;
    a.groups = G;
    a.g0 = 0;
    a.wire = w1;
    a.wire_lens = l1;
    a.status = s1;
    run_c(a);
    a.wire = w2;
    a.wire_lens = l2;
    a.status = s2;
    run_g(a);
    CK(hipDeviceSynchronize());
    std::vector<uint8_t> h1(G * n * slot), h2(G * n * slot);
    std::vector<uint16_t> hl1(G * n), hl2(G * n);
    std::vector<int8_t> hs1(G), hs2(G);
    CK(hipMemcpy(h1.data(), w1, h1.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(h2.data(), w2, h2.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(hl1.data(), l1, G * n * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hl2.data(), l2, G * n * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hs1.data(), s1, G, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hs2.data(), s2, G, hipMemcpyDeviceToHost));
    bool ok = h1 == h2 && hl1 == hl2 && hs1 == hs2;
    printf("{\"check\":\"k_tx_g == k_tx_c (wire, wire_lens, status; random lengths, header-only, bad)\","
           "\"same\":%s}\n", ok ? "true" : "false");
    if (!ok) return 2;
    CK(hipMemset(w2, 0x5c, G * n * slot));
    CK(hipMemset(l2, 0x77, G * n * 2));
    CK(hipMemset(s2, 0x33, G));
    run_cl(a);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h2.data(), w2, h2.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(hl2.data(), l2, G * n * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hs2.data(), s2, G, hipMemcpyDeviceToHost));
    ok = h1 == h2 && hl1 == hl2 && hs1 == hs2;
    printf("{\"check\":\"k_tx_c with the keystream in LDS == k_tx_c\",\"same\":%s}\n", ok ? "true" : "false");
    if (!ok) return 2;
    for (int swz = 0; swz < 2; ++swz) {
      CK(hipMemset(w2, 0x5c, G * n * slot));
      CK(hipMemset(l2, 0x77, G * n * 2));
      CK(hipMemset(s2, 0x33, G));
      run_o(a, swz);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(h2.data(), w2, h2.size(), hipMemcpyDeviceToHost));
      CK(hipMemcpy(hl2.data(), l2, G * n * 2, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hs2.data(), s2, G, hipMemcpyDeviceToHost));
      ok = h1 == h2 && hl1 == hl2 && hs1 == hs2;
      printf("{\"check\":\"k_tx_o<swz %d> == k_tx_c\",\"same\":%s}\n", swz, ok ? "true" : "false");
      if (!ok) return 2;
    }
    for (void* q : {(void*)dp, (void*)dl, (void*)w1, (void*)w2, (void*)l1, (void*)l2, (void*)s1, (void*)s2})
      CK(hipFree(q));
  }

  // ---- timing: 65,536 groups of 10 full packets, RC4, 3 rotated sets
  const uint64_t G = 65536;
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
    rot[r].groups = G;
    rot[r].g0 = 0;
  }
  const double bytes = double(G) * (d + n) * max_len;
  const uint64_t copy16 = static_cast<uint64_t>(bytes / 2) / 16;
  struct T {
    std::string name;
    std::function<void()> fn;
    std::vector<float> t;
  };
  int cnt = 0;
  std::vector<T> ts;
  ts.push_back({"k_tx_c (round 3 production)", [&] { run_c(rot[cnt++ % 3]); }, {}});
  ts.push_back({"k_tx_c, keystream staged in LDS per block", [&] { run_cl(rot[cnt++ % 3]); }, {}});
  ts.push_back({"k_tx_c LDS keystream, 3 blocks/CU (52 KiB LDS)", [&] { run_cl_cap(rot[cnt++ % 3], 52u * 1024u); }, {}});
  ts.push_back({"k_tx_c LDS keystream, 4 blocks/CU (39 KiB LDS)", [&] { run_cl_cap(rot[cnt++ % 3], 39u * 1024u); }, {}});
  ts.push_back({"k_tx_c LDS keystream, 1 block/CU (100 KiB LDS)", [&] { run_cl_cap(rot[cnt++ % 3], 100u * 1024u); }, {}});
  ts.push_back({"k_tx_c (round 3 production), again", [&] { run_c(rot[cnt++ % 3]); }, {}});
  ts.push_back({"k_tx_c, keystream staged in LDS per block, again", [&] { run_cl(rot[cnt++ % 3]); }, {}});
  // the copy reads and writes the wire buffers (G*13*1488 B each): the data
  // packets alone (G*10*1488 B) are smaller than half the bytes moved
  if (copy16 * 16 > G * n * slot) return 3;
  ts.push_back({"nt copy of the same bytes", [&] {
                  const int k = cnt++ % 3;
                  k_copy1<<<(copy16 + 255) / 256, 256>>>(reinterpret_cast<const u32x4*>(rot[k].wire),
                                                         reinterpret_cast<u32x4*>(rot[(k + 1) % 3].wire), copy16);
                }, {}});
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 6; ++w)
    for (auto& v : ts) v.fn();
  CK(hipDeviceSynchronize());
  const uint64_t fl16 = (768ull << 20) / 16;
  uint8_t* fl = nullptr;
  CK(hipMalloc(&fl, fl16 * 16));
  CK(hipMemset(fl, 1, fl16 * 16));
  for (int rr = 0; rr < rounds; ++rr)
    for (auto& v : ts) {
      k_flush<<<(fl16 + 255) / 256, 256>>>(reinterpret_cast<const u32x4*>(fl), reinterpret_cast<uint32_t*>(fl), fl16);
      CK(hipEventRecord(e0));
      for (int k = 0; k < 3; ++k) v.fn();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.t.push_back(ms * 1000.f / 3.f);
    }
  CK(hipGetLastError());
  for (auto& v : ts) {
    std::sort(v.t.begin(), v.t.end());
    const double med = v.t[v.t.size() / 2];
    printf("{\"variant\":\"%s\",\"groups\":%llu,\"median_us\":%.2f,\"min_us\":%.2f,\"GBps\":%.1f,\"frac\":%.4f}\n",
           v.name.c_str(), (unsigned long long)G, med, v.t[0], bytes / med / 1e3, bytes / med / 1e3 / 8000.0);
  }
  return 0;
}
