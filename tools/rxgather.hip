// rxgather.hip -- RX group assembly: the ring-ordered place kernel against the
// chunk path and the destination-ordered index + gather pair (rx_experiments.hpp), and the nt copy of
// the same bytes, cold regime (rotating rings and batches, a cache-evicting
// sweep before every sample), interleaved, medians.  Not product code.
//
// Ring: 65,536 groups of (10+3), 5% uniform loss, 1476-B packets in 1488-B
// slots, RC4 pad, planar [13][G][1472] batch (S = 1470), as
// tools/bench_host.py rx_case.  argv: rounds, order (shuffled | inorder).
// Every variant is first checked on the device against the production path on
// a ring with duplicates (different payloads), bad flags and short packets.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/rxgather tools/rxgather.hip
#include "../ugo_amd/csrc/rx_kernels.hip"
#include "rx_experiments.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

// nt copy of packet i's first 1472 bytes (92 chunks) to i*1472: the same
// bytes as RX moves, read from the slots, written densely.  4 chunks per
// thread, loads first.
__global__ __launch_bounds__(256) void k_copy_slots(const uint8_t* src, uint8_t* dst, uint64_t npk) {
  const uint64_t nch = npk * 92;
  const uint64_t stride = gridDim.x * 256ull;
  for (uint64_t c0 = blockIdx.x * 256ull + threadIdx.x; c0 < nch; c0 += 4 * stride) {
    u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t c = c0 + k * stride;
      if (c < nch) {
        const uint64_t i = c / 92, m = c - i * 92;
        v[k] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + i * 1488 + 16 * m));
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t c = c0 + k * stride;
      if (c < nch) __builtin_nontemporal_store(v[k], reinterpret_cast<u32x4*>(dst + 16 * c));
    }
  }
}

// the same, one chunk per thread, full grid (the form of the 6.47 TB/s
// ceiling in profiles/r1/kvar_cold12_regime.jsonl)
__global__ __launch_bounds__(256) void k_copy_slots1(const uint8_t* src, uint8_t* dst, uint64_t npk) {
  const uint64_t c = blockIdx.x * 256ull + threadIdx.x;
  if (c >= npk * 92) return;
  const uint64_t i = c / 92, m = c - i * 92;
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + i * 1488 + 16 * m));
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst + 16 * c));
}

__global__ __launch_bounds__(256) void k_copy_flat1(const uint8_t* src, uint8_t* dst, uint64_t n16) {
  const uint64_t c = blockIdx.x * 256ull + threadIdx.x;
  if (c >= n16) return;
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src) + c);
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst) + c);
}

// PATTERNS (nt, no decryption / realignment / header work: the access shapes only)
// P2: packet i's 92 chunks -> its planar destination (scatter), one chunk per thread, full grid
__global__ __launch_bounds__(256) void k_pat_scatter1(const uint8_t* src, uint8_t* dst, const uint64_t* doff,
                                                      uint64_t npk) {
  const uint64_t c = blockIdx.x * 256ull + threadIdx.x;
  if (c >= npk * 92) return;
  const uint64_t i = c / 92, m = c - i * 92;
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + i * 1488 + 16 * m));
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst + doff[i] + 16 * m));
}
// P2r: P2 with what an index-driven RX lane would add -- the payload at byte 6 of the slot (two
// aligned loads, the second mostly an L1/L2 hit, funnel-shifted) and the keystream chunk XORed
// (a load per lane from a 1488-B pad, L1/L2-resident); the destination from the per-packet index
__global__ __launch_bounds__(256) void k_pat_scatter1r(const uint8_t* src, uint8_t* dst, const uint64_t* doff,
                                                       const uint8_t* pad, uint64_t npk) {
  const uint64_t c = blockIdx.x * 256ull + threadIdx.x;
  if (c >= npk * 92) return;
  const uint64_t i = c / 92, m = c - i * 92;
  const u32x4* sp = reinterpret_cast<const u32x4*>(src + i * 1488 + 16 * m);
  const u32x4 a = __builtin_nontemporal_load(sp), b = __builtin_nontemporal_load(sp + 1);
  const u32x4 k0 = *reinterpret_cast<const u32x4*>(pad + 16 * m), k1 = *reinterpret_cast<const u32x4*>(pad + 16 * m + 16);
  const u32x4 x = a ^ k0, y = b ^ k1;
  u32x4 v;  // bytes [6, 22) of the 32 loaded
  v.x = __builtin_amdgcn_alignbyte(x.y, x.x, 6);
  v.y = __builtin_amdgcn_alignbyte(x.z, x.y, 6);
  v.z = __builtin_amdgcn_alignbyte(x.w, x.z, 6);
  v.w = __builtin_amdgcn_alignbyte(y.x, x.w, 6);
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst + doff[i] + 16 * m));
}
// P3 (DENSE=false) / P4 (DENSE=true): production structure -- half a wave per packet, 3 chunks per
// lane loaded first, grid-stride over packet pairs, 2048 blocks -- to the scattered / dense destination
template <bool DENSE>
__global__ __launch_bounds__(256) void k_pat_half(const uint8_t* src, uint8_t* dst, const uint64_t* doff,
                                                  uint64_t npk) {
  const uint32_t lane = threadIdx.x & 63u, half = lane >> 5, hl = lane & 31u;
  const uint64_t wave = (blockIdx.x * 256ull + threadIdx.x) >> 6;
  const uint64_t nwaves = (gridDim.x * 256ull) >> 6;
  for (uint64_t i = 2 * wave + half; i < npk; i += 2 * nwaves) {
    u32x4 A[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const uint32_t m = 32u * q + hl;
      if (m < 92) A[q] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + i * 1488 + 16 * m));
    }
    uint8_t* d = dst + (DENSE ? i * 1472 : doff[i]);
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const uint32_t m = 32u * q + hl;
      if (m < 92) __builtin_nontemporal_store(A[q], reinterpret_cast<u32x4*>(d + 16 * m));
    }
  }
}
// P5: destination order (gather): chunk m of planar piece j = row*G + g <- packet sidx[j], one
// chunk per thread, full grid; lost pieces skipped
__global__ __launch_bounds__(256) void k_pat_gather1(const uint8_t* src, uint8_t* dst, const uint32_t* sidx,
                                                     uint64_t pieces) {
  const uint64_t c = blockIdx.x * 256ull + threadIdx.x;
  if (c >= pieces * 92) return;
  const uint64_t j = c / 92, m = c - j * 92;
  const uint32_t i = sidx[j];
  if (i == 0xffffffffu) return;
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + uint64_t(i) * 1488 + 16 * m));
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst + 16 * c));
}

__global__ __launch_bounds__(256) void k_flush(const u32x4* a, uint32_t* out, uint64_t n16) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i >= n16) return;
  const u32x4 v = a[i];
  if ((v.x ^ v.y ^ v.z ^ v.w) == 0x9e3779b9u) out[0] = v.x;
}

struct Ring {
  std::vector<uint8_t> wire;
  std::vector<uint16_t> lens;
  uint64_t npk;
};

static Ring make_ring(uint64_t G, uint32_t n, uint32_t d, uint32_t slot, const std::vector<uint8_t>& pad, bool shuffle,
                      bool junk, uint64_t seed) {
  std::mt19937_64 rng(seed);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  std::vector<uint32_t> seq;
  std::vector<uint8_t> kind;  // 0 normal, 1 bad flag, 2 short
  for (uint64_t s = 0; s < G * n; ++s) {
    if (U(rng) < 0.05) continue;
    seq.push_back(static_cast<uint32_t>(s));
    kind.push_back(0);
    if (junk && U(rng) < 0.05) {  // a later copy with another payload
      seq.push_back(static_cast<uint32_t>(s));
      kind.push_back(0);
    }
    if (junk && U(rng) < 0.01) {
      seq.push_back(static_cast<uint32_t>(s));
      kind.push_back(U(rng) < 0.5 ? 1 : 2);
    }
  }
  std::vector<uint64_t> order(seq.size());
  for (uint64_t i = 0; i < order.size(); ++i) order[i] = i;
  if (shuffle) std::shuffle(order.begin(), order.end(), rng);
  Ring r;
  r.npk = seq.size();
  r.wire.resize(r.npk * slot);
  r.lens.resize(r.npk);
  for (uint64_t k = 0; k < r.npk; ++k) {
    const uint64_t i = order[k];
    uint8_t* w = &r.wire[k * slot];
    for (uint32_t b = 0; b < slot; b += 8) {
      const uint64_t x = rng();
      memcpy(w + b, &x, std::min<uint32_t>(8, slot - b));
    }
    const uint32_t s = seq[i];
    const uint8_t h[6] = {uint8_t(s), uint8_t(s >> 8), uint8_t(s >> 16), uint8_t(s >> 24),
                          uint8_t(kind[i] == 1 ? 0x77 : (s % n < d ? 0xf1 : 0xf2)), 0};
    for (int j = 0; j < 6; ++j) w[j] = h[j] ^ pad[j];
    r.lens[k] = kind[i] == 2 ? 4 : (junk ? static_cast<uint16_t>(6 + rng() % 1471) : 1476);
  }
  return r;
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 15;
  const bool shuffle = !(argc > 2 && std::string(argv[2]) == "inorder");
  const uint32_t d = 10, n = 13, S = 1470;
  // RXG_SLOT: the ring's slot stride (default 1488 = round_up(1476, 16); 1536 puts every packet on
  // 128-B lines of its own).  The PATTERN / copy lines assume 1488.
  const uint32_t slot = getenv("RXG_SLOT") ? static_cast<uint32_t>(atoi(getenv("RXG_SLOT"))) : 1488u;
  // RXG_PITCH: the batch's row pitch (default 1472 = round_up(S, 16); 1536 puts every row piece on its own
  // 128-B lines)
  const uint32_t pitch = getenv("RXG_PITCH") ? static_cast<uint32_t>(atoi(getenv("RXG_PITCH"))) : 1472u;
  const uint64_t G = 65536;
  std::mt19937_64 prng(11);
  std::vector<uint8_t> pad(slot);
  for (auto& b : pad) b = static_cast<uint8_t>(prng());
  uint8_t* d_pad;
  CK(hipMalloc(&d_pad, slot));
  CK(hipMemcpy(d_pad, pad.data(), slot, hipMemcpyHostToDevice));
  uint32_t* d_stats;
  CK(hipMalloc(&d_stats, 64));
  uint32_t* d_scr;  // prev [G] u64 | claim / index words [G][n] u32 | dup flag
  CK(hipMalloc(&d_scr, G * 8 + G * n * 4 + 64));
  uint64_t* prev = reinterpret_cast<uint64_t*>(d_scr);
  uint32_t* win = reinterpret_cast<uint32_t*>(prev + G);
  uint32_t* dup = win + G * n;

  enum Kind { PROD, PROD_OLD, GATHER, CHUNK, FULL, SLOTS, HALF, P2K };
  struct Var {
    std::string name;
    Kind kind;
    int order, gt;
    uint32_t grid;
  };
  std::vector<Var> vars = {
      {"production (round 5): begin(+claim fill, fresh flag) + k_rx_place_h (16384 blocks, whole-chunk row tails) + gated claim/re-place", PROD, 0, 0, 0},
      {"full-grid half-wave k_rx_half (P3b shape, no length-dependent loads, whole-chunk row tails) + tally + gated claim/re-place", HALF, 0, 0, 0},
      {"production kernel, plain payload loads (nt stores)", PROD, 30, 0, 0},
      {"production kernel, contiguous packet runs per wave, nt loads", PROD, 31, 0, 0},
      {"production kernel, contiguous packet runs per wave, plain payload loads", PROD, 32, 0, 0},
      {"k_rx_half, plain payload loads", HALF, 1, 0, 0},
      {"k_rx_p2: P2 shape, one chunk per lane, scalar headers, keystream per lane + tally + gated claim/re-place", P2K, 0, 0, 0},
      {"round-4 second form: k_rx_place MODE 4 (ds_bpermute realignment, header load), 8192 blocks", PROD, 7, 0, 0},
      {"production kernel, 8192 blocks", PROD, 0, 0, 8192},
      {"production, gated claim / re-place on 1024 blocks", PROD, 40, 0, 0},
      {"production with the byte masks on every chunk (round-5 first form, TAILB 0)", PROD, 42, 0, 0},
      {"production, claim words filled by a gated pass (not by begin), gated passes on 1024 blocks", PROD, 41, 0, 0},
      {"production (round 3): begin + place (MODE 0, 2048 blocks) + gated fill/claim/re-place", PROD_OLD, 0, 0, 2048},
      {"production with the place kernel's presence atomics removed (MODE 1, timing only)", PROD, 1, 0, 0},
      {"production with the place kernel's realignment removed (MODE 2, timing only)", PROD, 2, 0, 0},
  };
  if (const char* only = getenv("RXG_ONLY")) {  // the production form plus the variants whose name holds `only`
    std::vector<Var> keep = {vars[0]};
    for (size_t k = 1; k < vars.size(); ++k)
      if (vars[k].name.find(only) != std::string::npos) keep.push_back(vars[k]);
    vars = keep;
  }
  uint32_t* d_cnt;
  CK(hipMalloc(&d_cnt, kRxCntWords * 4));
  unsigned long long* d_seen;
  CK(hipMalloc(&d_seen, 8));
  CK(hipMemset(d_seen, 0, 8));
  unsigned long long call_id = 0;
  uint32_t* d_parts;
  CK(hipMalloc(&d_parts, (G * n + 7) / 8 * 5 * 4 + 64));
  auto full_grid = [&](const Var& v, const RxArgs& a) -> uint32_t {
    if (v.grid > 8) return v.grid;
    if (v.order == 0) return static_cast<uint32_t>((a.groups * n + 8 * v.grid - 1) / (8 * v.grid));
    return static_cast<uint32_t>((a.groups + v.gt - 1) / v.gt);
  };
  auto run = [&](const Var& v, RxArgs a, hipStream_t s, bool zero_present = true) {
    a.win = nullptr;
    a.prev = nullptr;
    a.dup = nullptr;
    a.gate = nullptr;
    a.fixup = 0;
    if (zero_present) CK(hipMemsetAsync(a.present, 0, a.groups * 8, s));
    a.seen = nullptr;
    a.call = 0;
    if (v.kind == GATHER) {
      CK(launch_rx_fill(win, a.groups * n, nullptr, s));
      a.win = win;
      const uint32_t ib = static_cast<uint32_t>((a.npk + 1023) / 1024);
      k_rx_index<4><<<ib, 256, 0, s>>>(a, d_parts);
      const uint32_t gr = full_grid(v, a);
      if (v.order == 0)
        k_rx_gather<3, 0, 1><<<gr, 256, 0, s>>>(a, d_parts, ib);
      else if (v.gt == 8)
        k_rx_gather<3, 1, 8><<<gr, 256, 0, s>>>(a, d_parts, ib);
      else
        k_rx_gather<3, 1, 32><<<gr, 256, 0, s>>>(a, d_parts, ib);
      return;
    }
    if (v.kind == SLOTS || v.kind == HALF || v.kind == P2K) {  // round 5: begin -> zero ctl -> place -> tally -> gated claim / re-place
      const unsigned long long call = ++call_id;
      CK(launch_rx_begin(a.present, prev, a.groups, dup, win, a.groups * n, d_seen, call, s));
      k_rx_zero_rare<<<1, 64, 0, s>>>(dup);  // ctl = dup[0..7] (ctl[0] is the duplicate gate)
      a.seen = d_seen;
      a.call = call;
      a.prev = prev;
      if (v.kind == HALF) {
        if (v.order == 1)
          k_rx_half<3, 0, 0, 0><<<static_cast<uint32_t>((a.npk + 7) / 8), 256, 0, s>>>(a, dup);
        else
          k_rx_half<3, 0><<<static_cast<uint32_t>((a.npk + 7) / 8), 256, 0, s>>>(a, dup);
      } else if (v.kind == P2K) {
        const uint64_t waves = (a.npk * (a.slot / 16) + 62) / 63;
        const uint32_t blocks = static_cast<uint32_t>((waves + 3) / 4);
        if (v.order == 1)
          k_rx_p2<1><<<blocks, 256, 0, s>>>(a, dup);
        else if (v.order == 2)
          k_rx_p2<0, 1><<<blocks, 256, 0, s>>>(a, dup);
        else
          k_rx_p2<0><<<blocks, 256, 0, s>>>(a, dup);
      } else {
        const uint64_t Q = a.slot / 16, nq = (a.S + 15) / 16, T = Q > nq ? Q : nq;
        uint32_t P = static_cast<uint32_t>(v.order);
        if (P * T > 1024) P = static_cast<uint32_t>(1024 / T);
        const uint32_t blocks = static_cast<uint32_t>((a.npk + P - 1) / P);
        const uint32_t shmem = static_cast<uint32_t>(16 * Q + P * 16 + P * T * 8);
        k_rx_slots<1><<<blocks, static_cast<uint32_t>(P * T), shmem, s>>>(a, static_cast<uint32_t>(T), P, dup);
      }
      uint64_t tb = (a.groups + 255) / 256;
      if (tb > 64u) tb = 64u;
      k_rx_tally<<<static_cast<uint32_t>(tb), 256, 0, s>>>(a.present, prev, a.groups, dup, a.stats, a.npk);
      RxArgs f = a;
      f.win = win;
      f.gate = dup;
      f.dup = nullptr;
      f.stats = nullptr;
      f.fixup = 1;
      CK(launch_rx_claim(f, s));
      CK(launch_rx_scatter(f, s));
      return;
    }
    if (v.kind == FULL) {
      CK(launch_rx_full_path(a, prev, win, dup, d_cnt, d_seen, ++call_id, s));
      return;
    }
    if (v.kind == CHUNK) {  // the round-4 chunk path (rx_experiments.hpp)
      CK(launch_rx_chunk_path(a, prev, win, dup, d_cnt, d_seen, ++call_id, s));
      return;
    }
    if (v.kind == PROD) {
      const unsigned long long call = ++call_id;
      if (v.order == 41)
        CK(launch_rx_begin(a.present, prev, a.groups, dup, nullptr, 0, d_seen, call, s));
      else
        CK(launch_rx_begin(a.present, prev, a.groups, dup, win, a.groups * n, d_seen, call, s));
      a.seen = d_seen;
      a.call = call;
    } else {
      CK(launch_rx_begin(a.present, prev, a.groups, dup, nullptr, 0, nullptr, 0, s));
    }
    a.dup = dup;
    a.prev = prev;
    const uint32_t blocks = v.grid ? v.grid : rx_blocks(a);
    if (v.kind == PROD && v.order == 42) {
      k_rx_place_h<3, 3, 0, 0><<<blocks, 256, 0, s>>>(a);
      RxArgs f = a;
      f.win = win;
      f.gate = dup;
      f.dup = nullptr;
      f.stats = nullptr;
      f.fixup = 1;
      CK(launch_rx_claim(f, s));
      k_rx_place_h<3, 3, 0, 0><<<1024, 256, 0, s>>>(f);
      return;
    }
    if (v.kind == PROD && (v.order == 40 || v.order == 41)) {
      k_rx_place_h<3, 3><<<blocks, 256, 0, s>>>(a);
      if (v.order == 41) CK(launch_rx_fill(win, a.groups * n, dup, s));
      RxArgs f = a;
      f.win = win;
      f.gate = dup;
      f.dup = nullptr;
      f.stats = nullptr;
      f.fixup = 1;
      k_rx_claim<<<1024, 256, 0, s>>>(f);
      k_rx_place_h<3, 3><<<1024, 256, 0, s>>>(f);
      return;
    }
    if (v.kind == PROD && (v.order == 0 || v.order == 5)) {
      if (v.order == 5)
        k_rx_place<3, 0, 3><<<blocks, 256, 0, s>>>(a);
      else
        k_rx_place_h<3, 3><<<blocks, 256, 0, s>>>(a);  // production
    } else if (v.kind == PROD && v.order == 30)
      k_rx_place_h<3, 2><<<blocks, 256, 0, s>>>(a);
    else if (v.kind == PROD && v.order == 31)
      k_rx_place_h<3, 3, 1><<<blocks, 256, 0, s>>>(a);
    else if (v.kind == PROD && v.order == 32)
      k_rx_place_h<3, 2, 1><<<blocks, 256, 0, s>>>(a);
    else if (v.kind == PROD && v.order == 7)
      k_rx_place<3, 4, 3><<<blocks, 256, 0, s>>>(a);
    else if (v.kind == PROD && v.order == 1)
      k_rx_place<3, 1, 3><<<blocks, 256, 0, s>>>(a);
    else if (v.kind == PROD && v.order == 2)
      k_rx_place<3, 2, 3><<<blocks, 256, 0, s>>>(a);
    else if (v.kind == PROD && v.order == 3)
      k_rx_place<3, 3, 3><<<blocks, 256, 0, s>>>(a);
    else
      k_rx_place<3, 0, 3><<<blocks, 256, 0, s>>>(a);
    if (v.kind == PROD_OLD) CK(launch_rx_fill(win, a.groups * n, dup, s));
    RxArgs f = a;
    f.win = win;
    f.gate = dup;
    f.dup = nullptr;
    f.stats = nullptr;
    f.fixup = 1;
    CK(launch_rx_claim(f, s));
    if (v.kind == PROD && v.order == 0)
      CK(launch_rx_scatter(f, s));  // production's re-place
    else
      k_rx_place<3, 0, 3><<<blocks, 256, 0, s>>>(f);
  };

  // ---- correctness: every variant against production on a ring with duplicates and junk
  {
    const uint64_t Gv = 4096;
    for (int sh = 0; sh < 4; ++sh) {
      const bool two = sh >= 2;
      Ring r = make_ring(Gv, n, d, slot, pad, (sh & 1) == 1, true, 99 + sh);
      uint8_t *w, *b;
      uint16_t* l;
      uint64_t* pres;
      CK(hipMalloc(&w, r.wire.size()));
      CK(hipMalloc(&l, r.npk * 2));
      CK(hipMalloc(&b, n * Gv * pitch));
      CK(hipMalloc(&pres, Gv * 8));
      CK(hipMemcpy(w, r.wire.data(), r.wire.size(), hipMemcpyHostToDevice));
      CK(hipMemcpy(l, r.lens.data(), r.npk * 2, hipMemcpyHostToDevice));
      RxArgs a{};
      a.wire = w; a.lens = l; a.pad = d_pad; a.shards = b; a.present = pres; a.stats = d_stats;
      a.npk = r.npk; a.slot = slot; a.first_group = 0; a.groups = Gv; a.rstride = Gv * pitch; a.gstride = pitch;
      a.S = S; a.n = n;
      std::vector<uint8_t> ref_b, got_b(n * Gv * pitch);
      std::vector<uint64_t> ref_p, got_p(Gv);
      std::vector<uint32_t> ref_s, got_s(5);
      for (size_t k = 0; k < vars.size(); ++k) {
        CK(hipMemset(b, 0xAB, n * Gv * pitch));
        CK(hipMemset(d_stats, 0, 64));
        if (two) {  // two calls into one batch: the second half of the ring second (non-fresh path)
          RxArgs a1 = a, a2 = a;
          a1.npk = r.npk / 2;
          a2.npk = r.npk - a1.npk;
          a2.wire = a.wire + a1.npk * slot;
          a2.lens = a.lens + a1.npk;
          run(vars[k], a1, nullptr, true);
          run(vars[k], a2, nullptr, false);
        } else {
          run(vars[k], a, nullptr);
        }
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(got_b.data(), b, got_b.size(), hipMemcpyDeviceToHost));
        CK(hipMemcpy(got_p.data(), pres, Gv * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(got_s.data(), d_stats, 20, hipMemcpyDeviceToHost));
        if (k == 0) {
          ref_b = got_b;
          ref_p = got_p;
          ref_s = got_s;
          printf("{\"check\":\"reference\",\"ring\":\"%s%s\",\"npk\":%llu,\"stats\":[%u,%u,%u,%u,%u]}\n",
                 (sh & 1) ? "shuffled" : "inorder", two ? " two calls" : "", (unsigned long long)r.npk, ref_s[0], ref_s[1], ref_s[2], ref_s[3], ref_s[4]);
          continue;
        }
        if (vars[k].kind == PROD && (vars[k].order == 1 || vars[k].order == 2)) continue;  // timing-only forms
        bool same_rows = true;  // bytes [0, S) of every row; the row tails past S are zero-filled since round 5
        for (size_t b = 0; b < got_b.size() && same_rows; ++b)
          if (b % pitch < S && got_b[b] != ref_b[b]) same_rows = false;
        const bool ok = same_rows && got_p == ref_p && got_s == ref_s;
        printf("{\"check\":\"%s\",\"ring\":\"%s%s\",\"same_as_production\":%s}\n", vars[k].name.c_str(),
               (sh & 1) ? "shuffled" : "inorder", two ? " two calls" : "", ok ? "true" : "false");
        if (!ok) return 2;
      }
      CK(hipFree(w)); CK(hipFree(l)); CK(hipFree(b)); CK(hipFree(pres));
    }
  }

  // ---- timing, cold: 3 rings / batches in rotation
  Ring r = make_ring(G, n, d, slot, pad, shuffle, false, 3);
  const uint64_t npk = r.npk;
  std::vector<RxArgs> rot(3);
  std::vector<uint8_t*> lin(3);
  for (int k = 0; k < 3; ++k) {
    uint8_t *w, *b;
    uint16_t* l;
    uint64_t* pres;
    CK(hipMalloc(&w, r.wire.size()));
    CK(hipMalloc(&l, npk * 2));
    CK(hipMalloc(&b, n * G * pitch));
    CK(hipMalloc(&pres, G * 8));
    CK(hipMalloc(&lin[k], npk * 1472));
    CK(hipMemcpy(w, r.wire.data(), r.wire.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(l, r.lens.data(), npk * 2, hipMemcpyHostToDevice));
    RxArgs a{};
    a.wire = w; a.lens = l; a.pad = d_pad; a.shards = b; a.present = pres; a.stats = d_stats;
    a.npk = npk; a.slot = slot; a.first_group = 0; a.groups = G; a.rstride = G * pitch; a.gstride = pitch;
    a.S = S; a.n = n;
    rot[k] = a;
  }
  // destination tables of the timing ring: planar offset per packet, packet per planar piece
  std::vector<uint64_t> doff(npk);
  std::vector<uint32_t> sidx(G * n, 0xffffffffu);
  for (uint64_t i = 0; i < npk; ++i) {
    uint32_t sq = 0;
    for (int j = 0; j < 4; ++j) sq |= uint32_t(r.wire[i * slot + j] ^ pad[j]) << (8 * j);
    const uint64_t row = sq % n, g = sq / n;
    doff[i] = row * G * pitch + g * pitch;
    sidx[row * G + g] = static_cast<uint32_t>(i);
  }
  uint64_t* d_doff;
  uint32_t* d_sidx;
  CK(hipMalloc(&d_doff, npk * 8));
  CK(hipMalloc(&d_sidx, G * n * 4));
  CK(hipMemcpy(d_doff, doff.data(), npk * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_sidx, sidx.data(), G * n * 4, hipMemcpyHostToDevice));
  uint8_t* d_padr;  // P2r's keystream (contents irrelevant to the timing)
  CK(hipMalloc(&d_padr, 1504));
  CK(hipMemset(d_padr, 0x5a, 1504));
  struct T {
    std::string name;
    std::function<void()> fn;
    std::vector<float> t;
  };
  std::vector<T> ts;
  int cnt = 0;
  ts.push_back({"nt copy of the same bytes (slots -> dense)", [&] {
                  const int k = cnt++ % 3;
                  k_copy_slots<<<4096, 256>>>(rot[k].wire, lin[k], npk);
                }, {}});
  ts.push_back({"nt copy of the same bytes, one chunk per thread, full grid", [&] {
                  const int k = cnt++ % 3;
                  k_copy_slots1<<<(npk * 92 + 255) / 256, 256>>>(rot[k].wire, lin[k], npk);
                }, {}});
  ts.push_back({"nt copy dense -> dense, same byte count, full grid", [&] {
                  const int k = cnt++ % 3;
                  k_copy_flat1<<<(npk * 92 + 255) / 256, 256>>>(rot[k].wire, lin[k], npk * 92);
                }, {}});
  ts.push_back({"PATTERN P2 scatter to planar, one chunk per thread, full grid", [&] {
                  const int k = cnt++ % 3;
                  k_pat_scatter1<<<(npk * 92 + 255) / 256, 256>>>(rot[k].wire, rot[k].shards, d_doff, npk);
                }, {}});
  ts.push_back({"PATTERN P2r: P2 + payload at byte 6 (two loads, funnel shift) + keystream XOR per lane", [&] {
                  const int k = cnt++ % 3;
                  k_pat_scatter1r<<<(npk * 92 + 255) / 256, 256>>>(rot[k].wire, rot[k].shards, d_doff, d_padr, npk);
                }, {}});
  ts.push_back({"PATTERN P3 scatter to planar, half-wave per packet, grid-stride 2048", [&] {
                  const int k = cnt++ % 3;
                  k_pat_half<false><<<2048, 256>>>(rot[k].wire, rot[k].shards, d_doff, npk);
                }, {}});
  ts.push_back({"PATTERN P4 dense, half-wave per packet, grid-stride 2048", [&] {
                  const int k = cnt++ % 3;
                  k_pat_half<true><<<2048, 256>>>(rot[k].wire, lin[k], d_doff, npk);
                }, {}});
  ts.push_back({"PATTERN P3b scatter to planar, half-wave per packet, full grid", [&] {
                  const int k = cnt++ % 3;
                  k_pat_half<false><<<(npk + 7) / 8, 256>>>(rot[k].wire, rot[k].shards, d_doff, npk);
                }, {}});
  ts.push_back({"PATTERN P5 gather in destination order, one chunk per thread, full grid", [&] {
                  const int k = cnt++ % 3;
                  k_pat_gather1<<<(G * n * 92 + 255) / 256, 256>>>(rot[k].wire, rot[k].shards, d_sidx, G * n);
                }, {}});
  for (const Var& v : vars) ts.push_back({v.name, [&, v] { run(v, rot[cnt++ % 3], nullptr); }, {}});
  ts.push_back({"chunk kernel alone, no returning atomic (timing bound; + memset present, begin)", [&] {
                  RxArgs a = rot[cnt++ % 3];
                  CK(hipMemsetAsync(a.present, 0, a.groups * 8, nullptr));
                  const unsigned long long call = ++call_id;
                  CK(launch_rx_begin(a.present, prev, a.groups, dup, win, a.groups * n, d_seen, call, nullptr));
                  k_rx_zero_cnt<<<1, 256>>>(d_cnt);
                  a.prev = prev;
                  a.seen = d_seen;
                  a.call = call;
                  a.dup = dup;
                  const uint64_t items = a.npk * 92;
                  k_rx_chunk<3, 0><<<(items + 255) / 256, 256>>>(a, 92, d_cnt);
                }, {}});
  ts.push_back({"index only (fill + index)", [&] {
                  RxArgs a = rot[cnt++ % 3];
                  a.win = win;
                  CK(hipMemsetAsync(a.present, 0, a.groups * 8, nullptr));
                  CK(launch_rx_fill(win, a.groups * n, nullptr, nullptr));
                  k_rx_index<4><<<(a.npk + 1023) / 1024, 256>>>(a, d_parts);
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
  const double bytes = double(npk) * (1476 + S);  // algorithmic: packet read + payload written
  for (auto& v : ts) {
    std::sort(v.t.begin(), v.t.end());
    const double med = v.t[v.t.size() / 2];
    printf("{\"variant\":\"%s\",\"ring\":\"%s\",\"pitch\":%u,\"packets\":%llu,\"median_us\":%.2f,\"min_us\":%.2f,"
           "\"GBps\":%.1f,\"frac\":%.4f,\"slot\":%u}\n",
           v.name.c_str(), shuffle ? "shuffled" : "inorder", pitch, (unsigned long long)npk, med, v.t[0],
           bytes / med / 1e3, bytes / med / 1e3 / 8000.0, slot);
  }
  return 0;
}
