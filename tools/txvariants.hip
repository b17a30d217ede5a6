// A/B timing of TX assembly kernel variants (store policy, scalar lengths).
// Not product code: includes the kernel TU.  Output: one JSON line per variant.
#include "../ugo_amd/csrc/tx_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <functional>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

using namespace ugo::kern;

// Compute-free TX pattern: the same 10 packet-chunk loads and 13 wire-chunk
// stores per thread as k_tx_c (full-length packets), parity = plain XORs.
template <int NTS>
__global__ __launch_bounds__(256) void k_tx_pattern(TxArgs a) {
  const uint32_t item = blockIdx.x * 256u + threadIdx.x;
  if (item >= a.groups * a.chunks) return;
  const uint64_t g = item / a.chunks;
  const uint32_t o = 16u * (item - static_cast<uint32_t>(g) * a.chunks);
  const uint8_t* src = a.pkts + g * 10 * a.slot_in + o;
  uint8_t* dst = a.wire + g * 13 * a.slot_out + o;
  V4 x[10];
#pragma unroll
  for (int k = 0; k < 10; ++k) x[k] = load16<1>(src + static_cast<uint64_t>(k) * a.slot_in);
#pragma unroll
  for (int k = 0; k < 10; ++k) store16<NTS>(dst + static_cast<uint64_t>(k) * a.slot_out, x[k], 16u);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    V4 y = x[i];
#pragma unroll
    for (int k = 3; k < 10; ++k)
      if ((k + i) & 1) xor4(y, x[k]);
    store16<NTS>(dst + static_cast<uint64_t>(10 + i) * a.slot_out, y, 16u);
  }
}

__global__ __launch_bounds__(256) void k_flush(const u32x4* a, uint32_t* out, uint64_t n16) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i >= n16) return;
  const u32x4 v = a[i];
  if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9e3779b9u) out[0] = v.x;
}

namespace ugo {
namespace kern {
LaunchTimer*& current_timer() {
  static thread_local LaunchTimer* t = nullptr;
  return t;
}
}  // namespace kern
}  // namespace ugo

int main(int argc, char** argv) {
  const uint64_t G = argc > 1 ? atoll(argv[1]) : 65536;
  const int rounds = argc > 2 ? atoi(argv[2]) : 11;
  const uint32_t d = 10, p = 3, n = 13, slot = 1488, maxl = 1476;
  uint8_t *pk, *wire, *pad;
  uint16_t *lens, *wl;
  CK(hipMalloc(&pk, G * d * slot));
  CK(hipMalloc(&wire, G * n * slot));
  CK(hipMalloc(&pad, slot));
  CK(hipMalloc(&lens, G * d * 2));
  CK(hipMalloc(&wl, G * n * 2));
  CK(hipMemset(pk, 0x3c, G * d * slot));
  CK(hipMemset(pad, 0x5a, slot));
  std::vector<uint16_t> hl(G * d, maxl);
  CK(hipMemcpy(lens, hl.data(), hl.size() * 2, hipMemcpyHostToDevice));
  TxArgs a{};
  a.pkts = pk; a.lens = lens; a.pad = pad; a.wire = wire; a.wire_lens = wl;
  a.groups = G; a.slot_in = slot; a.slot_out = slot; a.first_seq = 0; a.paws = (0xffffffffu / n - 1) * n;
  a.max_len = maxl; a.chunks = (maxl + 15) / 16; a.d = d; a.p = p; a.dpad = 12; a.epad = 4;
  const double bytes = double(G) * (2.0 * d * maxl + p * maxl);
  const uint32_t grid = (G * a.chunks + 255) / 256;
  struct Var { std::string name; std::function<void()> go; std::vector<float> t; };
  std::vector<Var> vars;
  auto add = [&](auto k, std::string nm) {
    vars.push_back({nm, [=]() { hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, a); }, {}});
  };
  add(k_tx_c<10, 3, 1, false>, "tx nt1 vector-lens");
  add(k_tx_c<10, 3, 1, true>, "tx nt1 scalar-lens");
  add(k_tx_c<10, 3, 3, false>, "tx nt3 vector-lens");
  add(k_tx_c<10, 3, 3, true>, "tx nt3 scalar-lens");
  add(k_tx_c<10, 3, 0, true>, "tx nt0 scalar-lens");
  // cold regime (argv[3] == "cold"): each launch on the next of 3 packet / wire buffer pairs
  std::vector<TxArgs> rot(3, a);
  int cnt = 0;
  if (argc > 3 && std::string(argv[3]) == "cold") {
    for (int r = 1; r < 3; ++r) {
      CK(hipMalloc(&rot[r].pkts, G * d * slot));
      CK(hipMemset(const_cast<uint8_t*>(rot[r].pkts), 0x3c, G * d * slot));
      CK(hipMalloc(&rot[r].wire, G * n * slot));
    }
    auto addc = [&](auto k, std::string nm) {
      vars.push_back({nm, [=, &rot, &cnt]() { hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, rot[cnt++ % 3]); }, {}});
    };
    addc(k_tx_c<10, 3, 0, false>, "COLD tx nt0");
    addc(k_tx_c<10, 3, 1, false>, "COLD tx nt1 (nt loads)");
    addc(k_tx_c<10, 3, 2, false>, "COLD tx nt2 (nt stores)");
    addc(k_tx_c<10, 3, 3, false>, "COLD tx nt3 (nt loads + stores)");
    addc(k_tx_pattern<0>, "COLD TX MEMORY PATTERN ONLY (nt loads, plain stores)");
    addc(k_tx_pattern<2>, "COLD TX MEMORY PATTERN ONLY (nt loads + stores)");
    // occupancy sweep (round 2): dynamic LDS caps the blocks per CU.  (Also
    // round 2, since removed: packets 0-7 or 0-9 by LDS-DMA at exactly 2 or 3
    // blocks/CU lose to production, 454.5 / 457.2 vs 447.5 us at 2 blocks,
    // profiles/r2/txvariants_ldsdma_exact_caps.jsonl.)
    for (uint32_t bpc : {4u, 3u, 2u}) {
      const uint32_t extra = 160u * 1024u / bpc + 512u;
      vars.push_back({"COLD OCC tx production (scalar lens, nt3), " + std::to_string(bpc) + " blocks/CU",
                      [=, &rot, &cnt]() {
                        hipLaunchKernelGGL((k_tx_c<10, 3, 3, true>), dim3(grid), dim3(256), extra, 0, rot[cnt++ % 3]);
                      }, {}});
    }
    vars.push_back({"COLD OCC tx production (scalar lens, nt3), natural occupancy", [=, &rot, &cnt]() {
      hipLaunchKernelGGL((k_tx_c<10, 3, 3, true>), dim3(grid), dim3(256), 0, 0, rot[cnt++ % 3]); }, {}});
    for (uint32_t bpc : {4u, 3u, 2u}) {
      const uint32_t extra = 160u * 1024u / bpc + 512u;
      vars.push_back({"COLD OCC TX MEMORY PATTERN ONLY (nt3), " + std::to_string(bpc) + " blocks/CU",
                      [=, &rot, &cnt]() {
                        hipLaunchKernelGGL((k_tx_pattern<2>), dim3(grid), dim3(256), extra, 0, rot[cnt++ % 3]);
                      }, {}});
    }
  }
  // correctness: every variant writes the same wire bytes
  std::vector<uint8_t> ref(G * n * slot), got(G * n * slot);
  for (size_t v = 0; v < 5; ++v) {
    CK(hipMemset(wire, 0, G * n * slot));
    vars[v].go();
    CK(hipMemcpy(v ? got.data() : ref.data(), wire, ref.size(), hipMemcpyDeviceToHost));
    if (v) printf("{\"check\":\"%s\",\"equal\":%s}\n", vars[v].name.c_str(), got == ref ? "true" : "false");
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // cold mode: an untimed 768-MB plain-load sweep before every sample evicts
  // the Infinity Cache (no sample pays for the previous one's dirty lines)
  const bool coldm = argc > 3 && std::string(argv[3]) == "cold";
  const uint64_t fl16 = (768ull << 20) / 16;
  uint8_t* fl = nullptr;
  if (coldm) {
    CK(hipMalloc(&fl, fl16 * 16));
    CK(hipMemset(fl, 1, fl16 * 16));
  }
  for (int r = 0; r < rounds; ++r)
    for (auto& v : vars) {
      if (coldm) hipLaunchKernelGGL(k_flush, dim3((fl16 + 255) / 256), dim3(256), 0, 0, reinterpret_cast<const u32x4*>(fl), reinterpret_cast<uint32_t*>(fl), fl16);
      CK(hipEventRecord(e0));
      for (int i = 0; i < 5; ++i) v.go();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.t.push_back(ms / 5);
    }
  for (auto& v : vars) {
    std::sort(v.t.begin(), v.t.end());
    const float med = v.t[v.t.size() / 2];
    printf("{\"variant\":\"%s\",\"median_us\":%.2f,\"min_us\":%.2f,\"GBps\":%.1f}\n", v.name.c_str(), med * 1e3,
           v.t[0] * 1e3, bytes / (med * 1e-3) / 1e9);
  }
  return 0;
}
