// ab_common.hpp -- shared by the A/B tools (kvariants.hip, bucket_probe.hip):
// the HIP error check and the host-built (10,3) MODE-1 descriptor table.
// Not product code; included after ../ugo_amd/csrc/fec_kernels.hip.
#pragma once
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));   \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

// canon: survivor slots aligned to row indices -- present data row r in slot r,
// the parity survivors in the erased data rows' slots (in order) -- so two
// groups sharing a wave load the same row in most slots.
static void build_table(int d, int p, uint32_t dpad, uint32_t epad, uint32_t stride, std::vector<uint8_t>& tab,
                        bool canon = false) {
  const int n = d + p;
  std::vector<uint8_t> M(n * d), scratch(n * d + 3 * d * d);
  gf::build_matrix(d, p, M.data(), scratch.data());
  tab.assign((size_t(1) << n) * stride + 64, 0);
  for (uint64_t m = 0; m < (1ull << n); ++m) {
    uint8_t* out = &tab[m * stride];
    int np = __builtin_popcountll(m);
    if (np == n) continue;
    if (np < d) { out[2] = 3; continue; }
    std::vector<int> surv, outr;
    for (int r = 0; r < n; ++r) {
      if ((m >> r) & 1) { if ((int)surv.size() < d) surv.push_back(r); } else outr.push_back(r);
    }
    std::vector<uint8_t> sub(d * d), inv(d * d), work(2 * d * d);
    for (int i = 0; i < d; ++i) memcpy(&sub[i * d], &M[surv[i] * d], d);
    gf::invert(d, sub.data(), inv.data(), work.data());
    int ed = 0;
    for (int r : outr) ed += r < d;
    out[0] = outr.size(); out[1] = ed;
    std::vector<int> slot(d);
    for (int k = 0; k < d; ++k) slot[k] = k;
    if (canon) {
      int nx = 0;
      std::vector<int> freeslots;
      for (int r = 0; r < d; ++r) if (!((m >> r) & 1)) freeslots.push_back(r);
      for (int k = 0; k < d; ++k) slot[k] = surv[k] < d ? surv[k] : freeslots[nx++];
    }
    for (int i = 0; i < d; ++i) out[4 + slot[i]] = surv[i];
    for (size_t i = 0; i < outr.size(); ++i) out[4 + dpad + i] = outr[i];
    uint8_t* coef = out + 4 + dpad + epad;
    for (size_t i = 0; i < outr.size(); ++i)
      for (int k = 0; k < d; ++k) {
        int r = outr[i];
        uint8_t v = 0;
        if (r < d) v = inv[r * d + k];
        else for (int j = 0; j < d; ++j) v ^= gf::mul(M[r * d + j], inv[j * d + k]);
        coef[i * dpad + slot[k]] = v;
      }
  }
}
