// tx_kernels.hip -- TX group assembly on gfx950.
//
// Replaces, for a whole batch of outgoing groups at once, the sender loop
// ugo/conn.go:643-685 (sendEncryptedData) and the per-packet encryption of
// Conn.sendPacket (ugo/conn.go:634):
//   markData(ori)                     LE32 next, LE16 0xf1 at [0,6)  ugo/fec.go:91-95
//   copy(fecGroup[k], ori); maxsize = max len
//   calcECC(fecGroup, 6, maxsize)     Encode of the window [6, maxsize) ugo/fec.go:228-243
//   markFEC(ecc[k]); ecc[k][:maxsize] LE32 next, LE16 0xf2, paws wrap ugo/fec.go:97-104
//   crypt.Encrypt(pkt, pkt)           fixed-key RC4 = XOR with one pad  ugo/crypto.go:33-39
//
// No realignment is needed: parity is column-independent, so a lane that
// holds *packet* bytes [16m, 16m+16) of every data packet (payload bytes
// [16m-6, 16m+10), header bytes zeroed) computes exactly the parity packet's
// bytes [16m, 16m+16).  Every load and store is an aligned 16-B chunk.
//
// Group buffers are zero-filled past each data packet's length (the reference
// loop reuses its 13 buffers without clearing them, so its parity bytes past a
// short packet depend on earlier groups; a fresh FEC -- or this batch -- sees
// zeros).  DESIGN.md §2 states this contract.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "gf_device.hpp"
#include "launch.hpp"
#include "tx_kernels.hpp"

namespace ugo {
namespace kern {

namespace {

constexpr uint32_t kTypeData = 0xf1u;  // ugo/constants.go:18
constexpr uint32_t kTypeFEC = 0xf2u;   // ugo/constants.go:19
constexpr int8_t kBadLength = 5;       // UGO_FEC_ERR_SHARD_SIZE
constexpr int8_t kNoData = 4;          // UGO_FEC_ERR_SHARD_NO_DATA
constexpr uint32_t kFecHeader = 6;     // fecHeaderSize, ugo/fec.go:11

__device__ __forceinline__ uint32_t keep_mask(uint32_t keep, int j) {
  const uint32_t lo = 4u * j;
  if (keep >= lo + 4u) return 0xffffffffu;
  if (keep <= lo) return 0u;
  return (1u << (8u * (keep - lo))) - 1u;
}

// bytes [keep, 16) of the chunk cleared (keep clamped to 0..16 by the masks)
__device__ __forceinline__ V4 keep_bytes(const V4& x, uint32_t keep) {
  V4 y;
#pragma unroll
  for (int j = 0; j < 4; ++j) y.v[j] = x.v[j] & keep_mask(keep, j);
  return y;
}

__device__ __forceinline__ void put_header(V4& x, uint32_t seq, uint32_t flag) {
  x.v[0] = seq;                                  // LE32 seqid
  x.v[1] = (x.v[1] & 0xffff0000u) | flag;        // LE16 flag
}

// launch policy (tools/txvariants.hip A/B, after the loads-first change):
// nontemporal loads and stores, lengths by scalar loads -- warm 484 us, cold
// 500 us (plain stores / vector lengths 490-507 us); the compute-free pattern
// of the same accesses is 454 us cold
constexpr int kTxNT = 3;
constexpr bool kTxSL = true;
// Data-packet loads: plain, not nontemporal (round 5).  A wave reads 1 KiB of
// each of a group's 10 packets, and slots of 1488 B put those spans' ends in
// the middle of 128-B lines that the neighbouring wave reads too: with
// nontemporal loads such a line was gone from L2 when the second wave asked,
// and was fetched again -- the 9 % of excess read bytes round 4 could not
// place (2 x FETCH_SIZE 1.0896 x the algorithmic bytes; plain loads 1.0656,
// and with XCD-contiguous blocks as well 1.0111).  Plain loads: 412.7 vs
// 455.0 us back to back, 413.0 vs 425.7 in interleaved cold rounds
// (tools/txpmc.hip, profiles/r5/txpmc_a/, txpmc_b/); the XCD-contiguous deal,
// despite its exact traffic, 451.9 / 452.0, and runs of 4 or 8 blocks per XCD
// (reads 0.96 / 0.955 of production's) 427.6 / 429.9 (txpmc_c/).
constexpr int kTxLoadNT = 0;

struct TxItem {
  uint64_t g;        // absolute group
  uint32_t o;        // packet byte offset of this lane's chunk
  uint32_t maxsz;    // parity packet length (max data packet length of the group)
  uint32_t seq0;     // seqid of the group's first packet
  V4 padc;
  bool live;
};

// Lengths, status, data packets out.  x[k] receives the parity inputs
// (packet chunk, bytes past the length and the header bytes zeroed).
//
// SL (even DN == d only): the lengths are read with scalar loads for the two
// groups a wave can span (>= 64 chunks per group) and picked per lane, instead
// of one broadcast vector load per packet per wave.
// ATTR (A/B and PMC attribution only, tools/txpmc.hip; 0 in production): bit 0
// skips the wire_lens / status stores, bit 1 replaces the parity network by a
// plain XOR of the inputs (the compute-free twin: wrong parity on purpose),
// bit 2 deals the blocks XCD-contiguously (consecutive blocks share one L2),
// bit 3 loads the data packets nontemporally (the round-4 policy), bit 4 / 5
// deal runs of 4 / 8 consecutive blocks to one XCD within windows of 32 / 64
// blocks (neighbours share an L2, the XCDs stay on nearby addresses).
template <int DN, int NT, bool SL, bool PL = false, int ATTR = 0>
__device__ __forceinline__ TxItem tx_data(const TxArgs& a, uint32_t item, V4* x, const u32x4* padl = nullptr) {
  TxItem t{};
  const uint64_t gl = item / a.chunks;
  const uint32_t m = item - static_cast<uint32_t>(gl) * a.chunks;
  t.g = a.g0 + gl;
  t.o = 16u * m;
  uint32_t Ls[DN];
  if constexpr (SL) {
    static_assert(DN % 2 == 0, "scalar lengths need an even d");
    const uint32_t wfirst = __builtin_amdgcn_readfirstlane(item) & ~63u;
    const uint64_t items = a.groups * a.chunks;
    const uint64_t wlast = min(static_cast<uint64_t>(wfirst) + 63u, items - 1u);
    const uint64_t gA = a.g0 + wfirst / a.chunks;
    const uint64_t gB = a.g0 + wlast / a.chunks;  // gA or gA + 1, never past the batch
    const uint8_t* lA = reinterpret_cast<const uint8_t*>(a.lens + gA * DN);
    const uint8_t* lB = reinterpret_cast<const uint8_t*>(a.lens + gB * DN);
    const bool inB = t.g != gA;
#pragma unroll
    for (int w = 0; w < DN / 2; ++w) {
      const uint32_t wa = ld32(lA + 4 * w), wb = ld32(lB + 4 * w);
      const uint32_t v = inB ? wb : wa;
      Ls[2 * w] = v & 0xffffu;
      Ls[2 * w + 1] = v >> 16;
    }
  } else {
    const uint16_t* L = a.lens + t.g * a.d;
#pragma unroll
    for (int k = 0; k < DN; ++k) Ls[k] = k < static_cast<int>(a.d) ? L[k] : 6u;
  }
  bool bad = false;
  uint32_t maxsz = 0;
#pragma unroll
  for (int k = 0; k < DN; ++k) {
    bad |= Ls[k] < 6u || Ls[k] > a.max_len;
    maxsz = max(maxsz, Ls[k]);
  }
  const uint32_t n = a.d + a.p;
  if (bad) {
    if (m == 0) {
      if (a.status) a.status[t.g] = kBadLength;
      for (uint32_t r = 0; r < n; ++r) a.wire_lens[t.g * n + r] = 0;
    }
    t.live = false;
    return t;
  }
  t.maxsz = maxsz;
  t.live = t.o < maxsz;
  t.seq0 = static_cast<uint32_t>((uint64_t(a.first_seq) + t.g * n) % a.paws);
  if (!t.live) return t;
  if constexpr (PL) {  // the block's LDS copy of the keystream
    const u32x4 v = padl[m];
    t.padc = V4{{v.x, v.y, v.z, v.w}};
  } else {
    t.padc = a.pad ? load16<0>(a.pad + t.o) : V4{{0u, 0u, 0u, 0u}};
  }
  const uint8_t* src = a.pkts + t.g * a.d * a.slot_in + t.o;
  uint8_t* dst = a.wire + t.g * n * a.slot_out + t.o;
  // all loads first: the stores below may alias the packets as far as the
  // compiler knows, so a load placed after a store waits for it
#pragma unroll
  for (int k = 0; k < DN; ++k) {
    x[k] = V4{{0u, 0u, 0u, 0u}};
    if (k < static_cast<int>(a.d) && t.o < Ls[k])
      x[k] = load16<(ATTR & 8) ? 1 : kTxLoadNT>(src + static_cast<uint64_t>(k) * a.slot_in);
  }
#pragma unroll
  for (int k = 0; k < DN; ++k) {
    if (k < static_cast<int>(a.d)) {
      const uint32_t Lk = Ls[k];
      V4 v = keep_bytes(x[k], Lk - min(Lk, t.o));
      if (t.o < Lk) {
        V4 w = v;
        if (m == 0) put_header(w, t.seq0 + k, kTypeData);
        xor4(w, t.padc);
        store16<NT>(dst + static_cast<uint64_t>(k) * a.slot_out, keep_bytes(w, Lk - t.o), 16u);
      }
      if (m == 0) {
        v.v[0] = 0u;
        v.v[1] &= 0xffff0000u;
        if constexpr (!(ATTR & 1)) a.wire_lens[t.g * n + k] = static_cast<uint16_t>(Lk);
      }
      x[k] = v;
    } else {
      x[k] = V4{{0u, 0u, 0u, 0u}};
    }
  }
  return t;
}

template <int NT, int ATTR = 0>
__device__ __forceinline__ void tx_parity_out(const TxArgs& a, const TxItem& t, uint32_t i, V4 y) {
  const uint32_t n = a.d + a.p;
  if (t.o == 0) put_header(y, t.seq0 + a.d + i, kTypeFEC);
  xor4(y, t.padc);
  store16<NT>(a.wire + (t.g * n + a.d + i) * a.slot_out + t.o, keep_bytes(y, t.maxsz - t.o), 16u);
  if constexpr (!(ATTR & 1))
    if (t.o == 0) a.wire_lens[t.g * n + a.d + i] = static_cast<uint16_t>(t.maxsz);
}

template <int D, int I>
__device__ __forceinline__ V4 xor_twin(const V4* x) {  // ATTR 2: the inputs XORed, rotated by the row
  V4 y = x[I % D];
#pragma unroll
  for (int k = 0; k < D; ++k)
    if (k != I % D) xor4(y, x[k]);
  return y;
}

template <int D, int P, int NT, int ATTR, int... I>
__device__ __forceinline__ void tx_cparity(const TxArgs& a, const TxItem& t, const V4* x,
                                           std::integer_sequence<int, I...>) {
  if constexpr (ATTR & 2)
    (tx_parity_out<NT, ATTR>(a, t, I, xor_twin<D, I>(x)), ...);
  else
    (tx_parity_out<NT, ATTR>(a, t, I, cparity<D, P, I>(x)), ...);
}

// Every data packet of the group header-only: calcECC's window [6, 6) is
// empty, its Encode fails (ErrShardNoData, ugo/fec.go:238-241) and the sender
// loop emits no parity packets (ugo/conn.go:669-673).  The group's data
// packets go out as usual; status UGO_FEC_ERR_SHARD_NO_DATA, parity wire_lens 0.
__device__ __forceinline__ bool tx_no_window(const TxArgs& a, const TxItem& t) {
  if (t.maxsz > kFecHeader) return false;
  if (t.o == 0) {
    if (a.status) a.status[t.g] = kNoData;
    const uint32_t n = a.d + a.p;
    for (uint32_t i = 0; i < a.p; ++i) a.wire_lens[t.g * n + a.d + i] = 0;
  }
  return true;
}

// (10,3) / (32,8): the compile-time XOR networks of k_encode_c.
// PL: the keystream staged once per block in dynamic LDS (needs a.pad and
// 16 * chunks bytes of dynamic LDS), instead of one 16-B global load per thread.
template <int RUN>
__device__ __forceinline__ uint32_t block_run() {  // hardware block b on XCD b % 8 -> runs of RUN logical blocks
  const uint32_t b = blockIdx.x, W = 8u * RUN;
  if (b >= gridDim.x / W * W) return b;
  return (b / W) * W + (b & 7u) * RUN + (b >> 3) % RUN;
}

template <int D, int P, int NT, bool SL, bool PL, int ATTR>
__device__ __forceinline__ void tx_c_item(const TxArgs& a, uint32_t item, const u32x4* padl) {
  V4 x[D];
  const TxItem t = tx_data<D, NT, SL, PL, ATTR>(a, item, x, padl);
  if (!t.live || tx_no_window(a, t)) return;
  tx_cparity<D, P, NT, ATTR>(a, t, x, std::make_integer_sequence<int, P>{});
  if constexpr (!(ATTR & 1))
    if (t.o == 0 && a.status) a.status[t.g] = 0;
}

// ATTR bit 6 (A/B only): a resident grid (2 blocks per CU) striding over the
// items instead of the full grid with its residency held by unused LDS.
template <int D, int P, int NT = kTxNT, bool SL = kTxSL, bool PL = false, int ATTR = 0>
__global__ __launch_bounds__(256) void k_tx_c(TxArgs a) {
  const uint32_t bid = (ATTR & 16) ? block_run<4>() : (ATTR & 32) ? block_run<8>() : block_id<(ATTR & 4) ? 1 : 0>();
  extern __shared__ u32x4 padl[];
  if constexpr (PL) {
    for (uint32_t i = threadIdx.x; i < a.chunks; i += 256u) padl[i] = *reinterpret_cast<const u32x4*>(a.pad + 16u * i);
    __syncthreads();
  }
  const uint32_t total = a.groups * a.chunks;
  if constexpr (ATTR & 64) {
    for (uint32_t base = bid * 256u; base < total; base += gridDim.x * 256u)
      if (base + threadIdx.x < total) tx_c_item<D, P, NT, SL, PL, ATTR>(a, base + threadIdx.x, padl);
  } else {
    const uint32_t item = bid * 256u + threadIdx.x;
    if (item >= total) return;
    tx_c_item<D, P, NT, SL, PL, ATTR>(a, item, padl);
  }
}

// Any other geometry: coefficients from the encode descriptor (uniform, so
// the coefficient words are scalar loads), masked Horner per parity row.
template <int DMAX, bool PL = false>
__global__ __launch_bounds__(256) void k_tx_var(TxArgs a) {
  const uint32_t item = blockIdx.x * 256u + threadIdx.x;
  extern __shared__ u32x4 padl[];
  if constexpr (PL) {  // the keystream staged once per block (as k_tx_c)
    for (uint32_t i = threadIdx.x; i < a.chunks; i += 256u) padl[i] = *reinterpret_cast<const u32x4*>(a.pad + 16u * i);
    __syncthreads();
  }
  if (item >= a.groups * a.chunks) return;
  V4 x[DMAX];
  const TxItem t = tx_data<DMAX, kTxNT, false, PL>(a, item, x, padl);
  if (!t.live || tx_no_window(a, t)) return;
  constexpr int NW = (DMAX + 3) / 4;
  const uint32_t cbase = 4 + a.dpad + a.epad;
  for (uint32_t i = 0; i < a.p; ++i) {
    uint32_t cw[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) cw[w] = ld32(a.desc + cbase + i * a.dpad + 4 * w);
    tx_parity_out<kTxNT>(a, t, i, horner_var<DMAX>(x, cw));
  }
  if (t.o == 0 && a.status) a.status[t.g] = 0;
}

}  // namespace

// Round 6 (VERDICT r5 follow-up): an LDS-staged form -- a block owning 1, 2
// or 4 whole groups, reading their data packets as one contiguous span into
// LDS, the parity columns from LDS, the wire packets out as one contiguous
// span (every line of a 4-group span whole) -- was bit-identical and ran
// 0.538-0.629 ms against this kernel's 0.455 on one box (256 / 512 threads,
// profiles/r6/tx_lds_ab.jsonl): the phases of a block serialize, and whole
// lines do not pay here (k_tx_c on 1536-B slots, every packet on lines of its
// own, ran 416 vs 413 us on 1488-B ones, profiles/r5/txpmc_b/).  Dropped.
// Residency cap for the (10,3) TX kernel: dynamic LDS it never touches limits
// it to 2 blocks (8 waves) per CU.  Fewer requests in flight run its 10-read +
// 13-write stream mix faster on a cold ring: 450.7 us at 2 blocks/CU, 464.6 at
// 3, 493.3 at its natural (VGPR-limited) occupancy, 567.5 at 1
// (tools/txvariants.hip, profiles/r2/txvariants_cold_occupancy.jsonl).  The
// cap is sized from the device's LDS per CU (half of it, less 1 KiB: 79 KiB
// on gfx950's 160 KiB), so it stays 2 blocks whatever the LDS size.  A
// waves-per-EU attribute only bounds the registers the compiler may use; it
// does not cap residency.
static uint32_t tx_lds_cap() {
  static const uint32_t cap = [] {
    int dev = 0, lds = 160 * 1024;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess ||
        lds <= 4096)
      lds = 160 * 1024;
    return static_cast<uint32_t>(lds / 2 - 1024);
  }();
  return cap;
}

hipError_t launch_tx_assemble(int dmax, const TxArgs& a, hipStream_t s) {
  const uint64_t items = a.groups * a.chunks;
  if (items == 0) return hipSuccess;
  const dim3 grid(static_cast<uint32_t>((items + 255) / 256)), block(256);
  switch (dmax) {
    case 0: {
      // scalar lengths need a wave to span at most 2 groups: >= 64 chunks per packet
      const bool sl = kTxSL && a.chunks >= 64;
      // with a keystream, each block stages it in LDS once (16 B per chunk;
      // the (10,3) kernel's residency cap already allocates far more): 424 vs
      // 439-445 us, one global load less per thread (tools/txgroup.hip,
      // profiles/r4/txgroup_pad_lds.jsonl)
      const uint32_t padl = 16u * a.chunks;
      const uint32_t cap = std::max(tx_lds_cap(), padl);
      // a block stages the whole keystream: only while that is at most one
      // group's worth of its 256 threads (chunks <= 256, max_len <= 4096) --
      // past that most of the stage goes unused and the lanes load
      // their own keystream chunk instead
      const bool pl = a.pad && a.chunks <= 256u;
      if (a.d == 10 && a.p == 3 && pl && sl)
        launch(kKTx, k_tx_c<10, 3, kTxNT, true, true>, grid, block, cap, s, a);
      else if (a.d == 10 && a.p == 3 && pl)
        launch(kKTx, k_tx_c<10, 3, kTxNT, false, true>, grid, block, cap, s, a);
      else if (a.d == 10 && a.p == 3 && sl)
        launch(kKTx, k_tx_c<10, 3, kTxNT, true>, grid, block, tx_lds_cap(), s, a);
      else if (a.d == 10 && a.p == 3)
        launch(kKTx, k_tx_c<10, 3, kTxNT, false>, grid, block, tx_lds_cap(), s, a);
      else if (a.d == 32 && a.p == 8 && pl && sl)
        launch(kKTx, k_tx_c<32, 8, kTxNT, true, true>, grid, block, padl, s, a);
      else if (a.d == 32 && a.p == 8 && pl)
        launch(kKTx, k_tx_c<32, 8, kTxNT, false, true>, grid, block, padl, s, a);
      else if (a.d == 32 && a.p == 8 && sl)
        launch(kKTx, k_tx_c<32, 8, kTxNT, true>, grid, block, 0, s, a);
      else if (a.d == 32 && a.p == 8)
        launch(kKTx, k_tx_c<32, 8, kTxNT, false>, grid, block, 0, s, a);
      else
        return hipErrorInvalidValue;
      break;
    }
#define UGO_TX_VAR(DM)                                                                   \
  case DM:                                                                               \
    if (a.pad && a.chunks <= 256u)                                                       \
      launch(kKTx, k_tx_var<DM, true>, grid, block, 16u * a.chunks, s, a);               \
    else                                                                                 \
      launch(kKTx, k_tx_var<DM>, grid, block, 0, s, a);                                  \
    break;
    UGO_TX_VAR(4)
    UGO_TX_VAR(8)
    UGO_TX_VAR(10)
    UGO_TX_VAR(12)
    UGO_TX_VAR(16)
    UGO_TX_VAR(24)
    UGO_TX_VAR(32)
#undef UGO_TX_VAR
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace kern
}  // namespace ugo
