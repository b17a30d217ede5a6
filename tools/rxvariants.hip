// rxvariants.hip -- interleaved A/B timing of the RX group-assembly kernels
// against the memory patterns that bound them (one process, rounds x
// variants, median reported).  Synthetic batch as tools/bench_host.py rx_case:
// 65,536 groups of (10+3), 5% uniform loss, shuffled arrival, 1476-B packets in
// 1488-B slots, RC4 pad, planar [13][G][1472] output.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/rxvariants tools/rxvariants.hip
// Not product code: it includes the kernel TU to instantiate variants.
#include "../ugo_amd/csrc/rx_kernels.hip"
#include "rx_experiments.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <numeric>
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

// Pattern ceiling: packet i's first `len` bytes -> an aligned planar row
// (same scatter destinations, no realignment, no header work), 16 B per lane,
// one wave per packet.
__global__ __launch_bounds__(256) void k_copy_scatter(RxArgs a, const uint32_t* dst_row) {
  const uint64_t wave = (blockIdx.x * 256ull + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t nwaves = (gridDim.x * 256ull) >> 6;
  for (uint64_t i = wave; i < a.npk; i += nwaves) {
    const uint8_t* pk = a.wire + i * a.slot;
    uint8_t* dst = a.shards + static_cast<uint64_t>(dst_row[i]) * a.gstride;
    for (uint32_t o = 16u * lane; o + 16u <= a.S + 2u; o += 1024u)
      *reinterpret_cast<u32x4*>(dst + o) = ld16(pk + o);
  }
}

// Plain stream copy of the same byte count (slots in order -> rows in order).
__global__ __launch_bounds__(256) void k_copy_linear(const u32x4* src, u32x4* dst, uint64_t n16) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += gridDim.x * 256ull) dst[i] = src[i];
}

__global__ __launch_bounds__(256) void k_flush(const u32x4* a, uint32_t* out, uint64_t n16) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i >= n16) return;
  const u32x4 v = a[i];
  if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9e3779b9u) out[0] = v.x;
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 15;
  const uint32_t d = 10, n = 13, S = 1470, pitch = 1472, slot = 1488;
  const uint64_t G = 65536;
  std::mt19937_64 rng(3);
  std::vector<uint32_t> seq;
  std::uniform_real_distribution<double> U(0.0, 1.0);
  for (uint64_t s = 0; s < G * n; ++s)
    if (U(rng) >= 0.05) seq.push_back(static_cast<uint32_t>(s));
  std::shuffle(seq.begin(), seq.end(), rng);
  const uint64_t npk = seq.size();
  std::vector<uint8_t> pad(slot);
  for (auto& b : pad) b = static_cast<uint8_t>(rng());
  std::vector<uint8_t> wire(npk * slot);
  for (auto& b : wire) b = static_cast<uint8_t>(rng());
  std::vector<uint32_t> dst_row(npk);
  for (uint64_t i = 0; i < npk; ++i) {
    uint8_t h[6] = {uint8_t(seq[i]), uint8_t(seq[i] >> 8), uint8_t(seq[i] >> 16), uint8_t(seq[i] >> 24),
                    uint8_t(seq[i] % n < d ? 0xf1 : 0xf2), 0};
    for (int j = 0; j < 6; ++j) wire[i * slot + j] = h[j] ^ pad[j];
    dst_row[i] = (seq[i] % n) * static_cast<uint32_t>(G) + seq[i] / n;  // row-major rows of [13][G]
  }
  std::vector<uint16_t> lens(npk, 1476);
  uint8_t *d_wire, *d_pad, *d_sh, *d_lin;
  uint16_t* d_lens;
  uint64_t* d_present;
  uint32_t *d_stats, *d_row;
  CK(hipMalloc(&d_wire, wire.size()));
  CK(hipMalloc(&d_pad, slot));
  CK(hipMalloc(&d_sh, n * G * pitch + 64));
  CK(hipMalloc(&d_lin, npk * slot));
  CK(hipMalloc(&d_lens, npk * 2));
  CK(hipMalloc(&d_present, G * 8));
  CK(hipMalloc(&d_stats, 16));
  CK(hipMalloc(&d_row, npk * 4));
  CK(hipMemcpy(d_wire, wire.data(), wire.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(d_pad, pad.data(), slot, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_lens, lens.data(), npk * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_row, dst_row.data(), npk * 4, hipMemcpyHostToDevice));
  CK(hipMemset(d_stats, 0, 16));
  RxArgs a{};
  a.wire = d_wire; a.lens = d_lens; a.pad = d_pad; a.shards = d_sh; a.present = d_present; a.stats = d_stats;
  a.npk = npk; a.slot = slot; a.first_group = 0; a.groups = G; a.rstride = G * pitch; a.gstride = pitch;
  a.S = S; a.n = n;
  const uint32_t blocks = rx_blocks(a);
  const double bytes = double(npk) * (1476 + S);  // algorithmic: packet read + payload written

  struct V {
    std::string name;
    std::function<void()> fn;
    std::vector<float> t;
  };
  std::vector<V> vs;
  vs.push_back({"k_rx_scatter (per-pass load->store)", [&] { k_rx_scatter<<<blocks, 256>>>(a); }, {}});
  vs.push_back({"k_rx_place<3> production", [&] { k_rx_place<3, 0><<<blocks, 256>>>(a); }, {}});
  vs.push_back({"k_rx_place<3> no presence atomics", [&] { k_rx_place<3, 1><<<blocks, 256>>>(a); }, {}});
  vs.push_back({"k_rx_place<3> no realignment", [&] { k_rx_place<3, 2><<<blocks, 256>>>(a); }, {}});
  vs.push_back({"k_rx_place<3> grid x2", [&] { k_rx_place<3, 0><<<blocks * 2, 256>>>(a); }, {}});
  vs.push_back({"k_rx_place<3> grid /2", [&] { k_rx_place<3, 0><<<blocks / 2, 256>>>(a); }, {}});
  vs.push_back({"PATTERN: aligned scatter copy, wave/packet", [&] { k_copy_scatter<<<2048, 256>>>(a, d_row); }, {}});
  vs.push_back({"PATTERN: linear copy of the same bytes",
                [&] { k_copy_linear<<<4096, 256>>>(reinterpret_cast<const u32x4*>(d_wire), reinterpret_cast<u32x4*>(d_lin), npk * 1480 / 16); }, {}});
  // Cold regime (argv[2] == "cold"): every launch takes the next of 3 wire
  // rings and 3 batches, so none of its lines are in the Infinity Cache.
  std::vector<RxArgs> rot(3, a);
  std::vector<uint8_t*> lin(3, d_lin);
  int cnt = 0;
  auto nx = [&]() -> const RxArgs& { return rot[cnt++ % 3]; };
  if (argc > 2 && std::string(argv[2]) == "cold") {
    vs.clear();
    for (int r = 1; r < 3; ++r) {
      uint8_t *w2, *s2, *l2;
      CK(hipMalloc(&w2, wire.size()));
      CK(hipMalloc(&s2, n * G * pitch + 64));
      CK(hipMalloc(&l2, npk * slot));
      CK(hipMemcpy(w2, d_wire, wire.size(), hipMemcpyDeviceToDevice));
      rot[r].wire = w2;
      rot[r].shards = s2;
      lin[r] = l2;
    }
    vs.push_back({"COLD k_rx_place<3> plain loads + stores", [&] { k_rx_place<3, 0, 0><<<blocks, 256>>>(nx()); }, {}});
    vs.push_back({"COLD k_rx_place<3> nt loads", [&] { k_rx_place<3, 0, 1><<<blocks, 256>>>(nx()); }, {}});
    vs.push_back({"COLD k_rx_place<3> nt stores", [&] { k_rx_place<3, 0, 2><<<blocks, 256>>>(nx()); }, {}});
    vs.push_back({"COLD k_rx_place<3> nt loads + stores", [&] { k_rx_place<3, 0, 3><<<blocks, 256>>>(nx()); }, {}});
    // occupancy (round 2): grid size (blocks per CU of the grid-stride loop) and LDS-capped residency
    for (uint32_t bpc : {8u, 6u, 4u, 3u}) {
      const uint32_t gb = 256u * bpc;
      vs.push_back({"COLD OCC k_rx_place<3> nt3, grid " + std::to_string(bpc) + " blocks/CU",
                    [&, gb] { k_rx_place<3, 0, 3><<<gb, 256>>>(nx()); }, {}});
    }
    for (uint32_t bpc : {6u, 4u}) {
      const uint32_t extra = 160u * 1024u / bpc + 512u;
      vs.push_back({"COLD OCC k_rx_place<3> nt3, grid 8/CU, LDS-capped at " + std::to_string(bpc) + " blocks/CU",
                    [&, extra] { k_rx_place<3, 0, 3><<<2048, 256, extra>>>(nx()); }, {}});
    }
    vs.push_back({"COLD PATTERN: linear copy of the same bytes", [&] {
      const int r = cnt++ % 3;
      k_copy_linear<<<4096, 256>>>(reinterpret_cast<const u32x4*>(rot[r].wire), reinterpret_cast<u32x4*>(lin[r]), npk * 1480 / 16); }, {}});
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 20; ++w)
    for (auto& v : vs) v.fn();
  CK(hipDeviceSynchronize());
  // cold mode: an untimed 768-MB plain-load sweep before every sample evicts
  // the Infinity Cache (no sample pays for the previous one's dirty lines)
  const bool coldm = argc > 2 && std::string(argv[2]) == "cold";
  const uint64_t fl16 = (768ull << 20) / 16;
  uint8_t* fl = nullptr;
  if (coldm) {
    CK(hipMalloc(&fl, fl16 * 16));
    CK(hipMemset(fl, 1, fl16 * 16));
  }
  for (int r = 0; r < rounds; ++r)
    for (auto& v : vs) {
      if (coldm) k_flush<<<(fl16 + 255) / 256, 256>>>(reinterpret_cast<const u32x4*>(fl), reinterpret_cast<uint32_t*>(fl), fl16);
      CK(hipEventRecord(e0));
      for (int k = 0; k < 5; ++k) v.fn();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.t.push_back(ms * 1000.f / 5.f);
    }
  CK(hipGetLastError());
  for (auto& v : vs) {
    std::sort(v.t.begin(), v.t.end());
    const double med = v.t[v.t.size() / 2];
    printf("{\"variant\":\"%s\",\"packets\":%llu,\"median_us\":%.2f,\"min_us\":%.2f,\"GBps\":%.1f}\n", v.name.c_str(),
           (unsigned long long)npk, med, v.t[0], bytes / med / 1e3);
  }
  return 0;
}
