// A/B timing of the (32,8) jumbo TX assembly: production k_tx_c (Horner
// network) against k_tx_fr (Four-Russians network), 8,192 groups of full
// 9006-B packets, RC4 pad.  Every variant's wire output (packets + lengths)
// must equal production's.  Not product code: includes the kernel TU.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/txjvariants tools/txjvariants.hip
#include "../ugo_amd/csrc/tx_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

using namespace ugo::kern;

namespace ugo {
namespace kern {
namespace {
// k_tx_c with the Four-Russians network (gf_device.hpp cparity_fr_seq, all
// rows from registers).  A/B only: it ties production (1151 vs 1146 us).
template <int D, int P, int NT = kTxNT, bool SL = kTxSL, int WPE = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_tx_fr(TxArgs a) {
  const uint32_t item = blockIdx.x * 256u + threadIdx.x;
  if (item >= a.groups * a.chunks) return;
  V4 x[D];
  const TxItem t = tx_data<D, NT, SL>(a, item, x);
  if (!t.live || tx_no_window(a, t)) return;
  V4 y[P];
  cparity_fr_seq<D, P, 0>(y, x, nullptr);
#pragma unroll
  for (int i = 0; i < P; ++i) tx_parity_out<NT>(a, t, i, y[i]);
  if (t.o == 0 && a.status) a.status[t.g] = 0;
}

}  // namespace
}  // namespace kern
}  // namespace ugo

namespace ugo {
namespace kern {
LaunchTimer*& current_timer() {
  static thread_local LaunchTimer* t = nullptr;
  return t;
}
}  // namespace kern
}  // namespace ugo

int main(int argc, char** argv) {
  const uint64_t G = argc > 1 ? atoll(argv[1]) : 8192;
  const int rounds = argc > 2 ? atoi(argv[2]) : 9;
  const uint32_t d = 32, p = 8, n = 40, maxl = 9006, slot = (maxl + 15) / 16 * 16;
  uint8_t *pk, *wire, *pad;
  uint16_t *lens, *wl;
  CK(hipMalloc(&pk, G * d * slot));
  CK(hipMalloc(&wire, G * n * slot));
  CK(hipMalloc(&pad, slot));
  CK(hipMalloc(&lens, G * d * 2));
  CK(hipMalloc(&wl, G * n * 2));
  {
    std::vector<uint8_t> h(G * d * slot);
    uint64_t st = 0x5EED;
    for (auto& b : h) { st = st * 6364136223846793005ull + 1442695040888963407ull; b = st >> 56; }
    CK(hipMemcpy(pk, h.data(), h.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(pad, h.data() + 12345, slot, hipMemcpyHostToDevice));
  }
  std::vector<uint16_t> hl(G * d, maxl);
  CK(hipMemcpy(lens, hl.data(), hl.size() * 2, hipMemcpyHostToDevice));
  TxArgs a{};
  a.pkts = pk; a.lens = lens; a.pad = pad; a.wire = wire; a.wire_lens = wl;
  a.groups = G; a.slot_in = slot; a.slot_out = slot; a.first_seq = 0; a.paws = (0xffffffffu / n - 1) * n;
  a.max_len = maxl; a.chunks = slot / 16; a.d = d; a.p = p; a.dpad = 32; a.epad = 8;
  const double bytes = double(G) * (2.0 * d * maxl + p * maxl);
  const uint32_t grid = (G * a.chunks + 255) / 256;
  struct Var { std::string name; std::function<void()> go; std::vector<float> t; };
  std::vector<Var> vars;
  auto add = [&](auto k, std::string nm) {
    vars.push_back({nm, [=]() { hipLaunchKernelGGL(k, dim3(grid), dim3(256), 0, 0, a); }, {}});
  };
  add(k_tx_c<32, 8, kTxNT, true>, "tx (32,8) Horner network (production)");
  add(k_tx_fr<32, 8, kTxNT, true>, "tx (32,8) Four-Russians network");
  add(k_tx_fr<32, 8, kTxNT, true, 2>, "tx (32,8) Four-Russians network, 2 waves/SIMD");
  add(k_tx_fr<32, 8, kTxNT, true, 3>, "tx (32,8) Four-Russians network, 3 waves/SIMD");
  const size_t wbytes = G * n * slot;
  std::vector<uint8_t> ref(wbytes), got(wbytes);
  std::vector<uint16_t> rl(G * n), gl(G * n);
  CK(hipMemset(wire, 0, wbytes));
  vars[0].go();
  CK(hipMemcpy(ref.data(), wire, wbytes, hipMemcpyDeviceToHost));
  CK(hipMemcpy(rl.data(), wl, rl.size() * 2, hipMemcpyDeviceToHost));
  for (size_t v = 1; v < vars.size(); ++v) {
    CK(hipMemset(wire, 0, wbytes));
    CK(hipMemset(wl, 0, G * n * 2));
    vars[v].go();
    CK(hipMemcpy(got.data(), wire, wbytes, hipMemcpyDeviceToHost));
    CK(hipMemcpy(gl.data(), wl, gl.size() * 2, hipMemcpyDeviceToHost));
    printf("{\"check\":\"%s == production\",\"equal\":%s}\n", vars[v].name.c_str(),
           (ref == got && rl == gl) ? "true" : "false");
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& v : vars) v.go();
  CK(hipDeviceSynchronize());
  for (int r = 0; r < rounds; ++r)
    for (auto& v : vars) {
      CK(hipEventRecord(e0));
      for (int i = 0; i < 3; ++i) v.go();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.t.push_back(ms / 3);
    }
  for (auto& v : vars) {
    std::sort(v.t.begin(), v.t.end());
    const float med = v.t[v.t.size() / 2];
    printf("{\"variant\":\"%s\",\"median_us\":%.2f,\"min_us\":%.2f,\"GBps\":%.1f}\n", v.name.c_str(), med * 1e3,
           v.t[0] * 1e3, bytes / (med * 1e-3) / 1e9);
  }
  return 0;
}
