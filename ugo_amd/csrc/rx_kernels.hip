// rx_kernels.hip -- RX group assembly on gfx950.
//
// Replaces, for a whole batch of received packets at once, the per-packet
// work ugo does before Reconstruct:
//   Conn.handlePacket: crypt.Decrypt(data, data)        ugo/conn.go:390
//     rc4StreamCrypto.Decrypt builds a fresh RC4 cipher per packet from a
//     fixed key (ugo/crypto.go:33-39), so decryption is an XOR with one
//     constant keystream prefix -> fused here as XOR with `pad`.
//   FEC.decode: LE32 seqid, LE16 flag, payload data[6:] ugo/fec.go:78-89
//   FEC.input: group = seqid - seqid % n, slot = seqid % n  ugo/fec.go:145,175
// Each packet lands in row seqid % n, group seqid / n - first_group of a
// strided (normally shard-major / planar) batch, zero-filled past its
// payload, and its presence bit is OR-ed into present[group]; Reconstruct
// (k_apply*) then runs over the batch.
//
// Duplicates: input drops a packet whose seqid is already queued, so the
// first arrival of a seqid is the one kept (ugo/fec.go:123-129).  A batch is
// filled by one or more calls, each a window of arrivals in ring order; the
// first copy wins, across calls as within one.  Across calls: the call's
// first launch snapshots the presence masks (8 B per group), and a packet
// whose bit was already set there belongs to a seqid an earlier call placed --
// it is a duplicate and writes nothing.  Within a call the first copy in ring
// order must win.  Duplicates are rare, so placement is optimistic: the place kernel
// writes every accepted packet and learns from its presence atomicOr whether
// the (group, row) was already taken; if any was, a flag is set and three
// gated kernels -- which return at once when it is not -- fill the claim
// words, take per (group, row) the smallest packet index (atomicMin,
// k_rx_claim) and re-place exactly the winners over whatever the racing
// copies left.  Without duplicates that costs three empty launches instead of
// a claim pass over every header before placement (DESIGN_HISTORY.md §4).
//
// The packet sits at a 16-aligned slot, so its payload (offset 6) is
// misaligned: each thread loads the two aligned chunks covering its 16 output
// bytes, XORs the keystream chunks, and realigns with v_alignbyte.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "launch.hpp"
#include "rx_kernels.hpp"

namespace ugo {
namespace kern {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 ld16(const uint8_t* p) { return *reinterpret_cast<const u32x4*>(p); }

__device__ __forceinline__ uint32_t from_next_lane(uint32_t v) {
  // DPP wave_shl:1 -- lane l receives lane l+1's value (lane 63 receives 0)
  return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(v), 0x130, 0xf, 0xf, false));
}

// Each half-wave owns one packet at a time (2 packets per wave-iteration);
// its 32 lanes cover the payload in passes of 32 chunks (92 chunks of a
// 1470-B payload -> 3 passes, 96% of lanes busy).  The second aligned chunk a
// lane needs for the realignment is its right neighbour's first chunk, taken
// with DPP instead of a second load (lane 31 of each half loads it).  The
// next packet's header is fetched before the current payload is processed.
// Measured alternatives: one wave per packet with two loads per chunk 1.4x
// slower; one thread per chunk across packets 4.5x slower (5 loads per 16 B).
// Presence bit, duplicate detection and stats of placed packets (lane 0 of
// each half-wave): the optimistic pass counts a packet whose bit was already
// set as a duplicate and raises a.dup; the re-place pass touches nothing.
// The presence atomicOr returns the old mask, and waiting for it inside the
// packet loop stalls the wave for a full memory round trip per packet (RX
// 512 vs ~470 us), so a packet's result is settled one iteration later.
struct RxAccount {
  unsigned long long old = 0;
  uint32_t why = 5, row = 0;
  __device__ __forceinline__ void settle(const RxArgs& a, uint32_t* bstats) {
    if (why >= 5) return;
    uint32_t w = why;
    if (w == 0 && a.dup && ((old >> row) & 1ull)) {
      w = 4;
      *a.dup = 1u;
    }
    atomicAdd(&bstats[w], 1u);
    why = 5;
  }
  __device__ __forceinline__ void issue(const RxArgs& a, uint32_t* bstats, uint32_t w, uint64_t gs, uint32_t r) {
    settle(a, bstats);
    if (a.fixup || w >= 5) return;
    why = w;
    row = r;
    old = 0;
    if (w == 0) old = atomicOr(reinterpret_cast<unsigned long long*>(&a.present[gs]), 1ull << r);
  }
};

__device__ __forceinline__ bool rx_gated_off(const RxArgs& a) { return a.gate && *a.gate == 0u; }

__global__ __launch_bounds__(256) void k_rx_scatter(RxArgs a) {
  if (rx_gated_off(a)) return;
  // stats: summed per block in LDS, one atomic per block per counter (a device
  // counter hit once per packet serialises at ~11 ns per atomic:
  // MI355X_MICROARCH.md "fanin")
  __shared__ uint32_t bstats[5];
  if (threadIdx.x < 5) bstats[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, half = lane >> 5, hl = lane & 31u;
  const uint64_t wave = (blockIdx.x * 256ull + threadIdx.x) >> 6;
  const uint64_t nwaves = (gridDim.x * 256ull) >> 6;
  const uint32_t nq = (a.S + 15u) / 16u;  // output chunks per row
  RxAccount acct;
  uint64_t i = 2 * wave + half;
  u32x4 hn = {0u, 0u, 0u, 0u};
  if (i < a.npk) hn = ld16(a.wire + i * a.slot);
  for (uint64_t base = 2 * wave; base < a.npk; base += 2 * nwaves, i += 2 * nwaves) {
    const bool have = i < a.npk;
    const uint8_t* pk = a.wire + i * a.slot;
    u32x4 h = hn;
    const uint64_t inext = i + 2 * nwaves;
    if (inext < a.npk) hn = ld16(a.wire + inext * a.slot);  // prefetch next header
    const uint32_t len = have ? a.lens[i] : 0u;
    if (a.pad) h ^= ld16(a.pad);
    const uint32_t seqid = h.x;
    const uint32_t flag = h.y & 0xffffu;
    uint32_t why = 0;  // 0 = accept, else stats slot (5: no packet)
    if (!have) why = 5;
    else if (len < 6u) why = 3;
    else if (flag != 0xf1u && flag != 0xf2u) why = 1;  // ugo/conn.go:395
    const uint32_t row = seqid % a.n;
    const uint64_t grp = seqid / a.n;
    if (!why && (grp < a.first_group || grp >= a.first_group + a.groups)) why = 2;
    const uint64_t gs = grp - a.first_group;
    if (!why && a.prev && ((a.prev[gs] >> row) & 1ull)) why = 4;  // placed by an earlier call
    if (!why && a.win && a.win[gs * a.n + row] != static_cast<uint32_t>(i)) why = 4;  // not the first copy
    const bool ok = why == 0;
    uint8_t* dst = a.shards + row * a.rstride + gs * a.gstride;
    const uint32_t L = ok ? min(len - 6u, a.S) : 0u;  // copy(buf, data[6:]) bounded by the row
    for (uint32_t q0 = 0; q0 < nq; q0 += 32u) {
      const uint32_t o = 16u * (q0 + hl);  // payload byte offset of this lane's chunk
      u32x4 A = {0u, 0u, 0u, 0u};
      if (o < L + 6u) {  // packet bytes [o, o+16) start inside the packet (the left
                         // neighbour needs them even when o >= payload length)
        A = ld16(pk + o);
        if (a.pad) A ^= ld16(a.pad + o);
      }
      // converged: neighbour's chunk (packet bytes [o+16, o+32)) by DPP
      uint32_t bx = from_next_lane(A.x), by = from_next_lane(A.y);
      if (hl == 31u && o + 16u < L + 6u && o + 16u < a.slot) {
        u32x4 B = ld16(pk + o + 16u);
        if (a.pad) B ^= ld16(a.pad + o + 16u);
        bx = B.x;
        by = B.y;
      }
      if (ok && o < a.S) {
        // payload bytes [o, o+16) = packet bytes [o+6, o+22)
        uint32_t w[4];
        w[0] = __builtin_amdgcn_alignbyte(A.z, A.y, 2);
        w[1] = __builtin_amdgcn_alignbyte(A.w, A.z, 2);
        w[2] = __builtin_amdgcn_alignbyte(bx, A.w, 2);
        w[3] = __builtin_amdgcn_alignbyte(by, bx, 2);
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // zero bytes past the payload
          const uint32_t b0 = o + 4u * j;
          const uint32_t keep = L >= b0 + 4u ? 4u : (L > b0 ? L - b0 : 0u);
          w[j] &= keep >= 4u ? 0xffffffffu : ((1u << (8u * keep)) - 1u);
        }
        const uint32_t nb = a.S - o;
        if (nb >= 16u) {
          *reinterpret_cast<u32x4*>(dst + o) = u32x4{w[0], w[1], w[2], w[3]};
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const uint32_t lo = 4u * j;
            if (nb >= lo + 4u) {
              *reinterpret_cast<uint32_t*>(dst + o + lo) = w[j];
            } else if (nb > lo) {
              for (uint32_t t = 0; t < nb - lo; ++t) dst[o + lo + t] = static_cast<uint8_t>(w[j] >> (8u * t));
            }
          }
        }
      }
    }
    if (hl == 0) acct.issue(a, bstats, why, gs, row);
  }
  if (hl == 0) acct.settle(a, bstats);
  if (a.stats) {
    __syncthreads();
    if (threadIdx.x < 5 && bstats[threadIdx.x]) atomicAdd(&a.stats[threadIdx.x], bstats[threadIdx.x]);
  }
}

// Loads-first form for rows of at most 32 * NP chunks (NP = 3 for ugo's
// 1470-B payloads).  Same decomposition (half a wave per packet), but:
//  * the keystream chunks at a lane's offsets are the same for every packet,
//    so they are loaded once and held in registers;
//  * the next packet's header and length are prefetched, so a packet's
//    placement is known before its payload arrives, and all NP payload loads of
//    a packet are issued before its first store (the per-pass load -> store
//    chain of k_rx_scatter kept one 1-KiB load in flight per wave);
//  * lengths are clamped to the slot.
// MODE (A/B timing only, tools/rxvariants.hip): 0 = production, 1 = without
// the presence atomics, 2 = the same loads and stores without the realignment.
// NT: bit 0 nontemporal payload loads, bit 1 nontemporal stores.
template <int NP, int MODE = 0, int NT = 0, int ORD = 0>
__global__ __launch_bounds__(256) void k_rx_place(RxArgs a) {
  if (rx_gated_off(a)) return;
  __shared__ uint32_t bstats[5];
  if (threadIdx.x < 5) bstats[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, half = lane >> 5, hl = lane & 31u;
  const uint64_t wave = (blockIdx.x * 256ull + threadIdx.x) >> 6;
  const uint64_t nwaves = (gridDim.x * 256ull) >> 6;
  const u32x4 zero = {0u, 0u, 0u, 0u};
  const uint32_t slot = static_cast<uint32_t>(a.slot);
  const u32x4 K0 = a.pad ? ld16(a.pad) : zero;  // keystream over the header chunk
  // a batch with no presence bit at call entry (the usual case: one call per
  // batch) has nothing an earlier call placed: no per-packet snapshot lookup
  const bool chk_prev = a.prev && !(a.seen && *a.seen < a.call);
  u32x4 K[NP];
  uint32_t kbx[NP], kby[NP];  // keystream of the neighbour chunk (lane 31 of a half)
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const uint32_t o = 16u * (32u * q + hl);
    K[q] = (a.pad && o + 16u <= slot) ? ld16(a.pad + o) : zero;
    kbx[q] = kby[q] = 0u;
    if (a.pad && hl == 31u && o + 32u <= slot) {
      const u32x4 B = ld16(a.pad + o + 16u);
      kbx[q] = B.x;
      kby[q] = B.y;
    }
  }
  RxAccount acct;
  // ORD 0: grid-stride over packet pairs.  ORD 1: block b owns the contiguous
  // packet range [b*per, b*per + per) (per a multiple of 8), its eight
  // half-waves take packets b*per + h, + 8, ...
  uint64_t first = 2 * wave, step = 2 * nwaves, end = a.npk;
  if constexpr (ORD == 1) {
    uint64_t per = (a.npk + gridDim.x - 1) / gridDim.x;
    per = (per + 7) / 8 * 8;
    first = blockIdx.x * per + 2 * (threadIdx.x >> 6);
    step = 8;
    end = min(a.npk, blockIdx.x * per + per);
  }
  uint64_t i = first + half;
  u32x4 hn = zero;
  uint32_t ln = 0;
  if (i < end) {
    hn = ld16(a.wire + i * a.slot);
    ln = a.lens[i];
  }
  for (uint64_t base = first; base < end; base += step, i += step) {
    const bool have = i < end;
    const uint8_t* pk = a.wire + i * a.slot;
    const u32x4 h = hn ^ K0;
    const uint32_t len = have ? min(ln, slot) : 0u;
    const uint64_t inext = i + step;
    if (inext < end) {  // prefetch the next packet's header and length
      hn = ld16(a.wire + inext * a.slot);
      ln = a.lens[inext];
    }
    const uint32_t seqid = h.x;
    const uint32_t flag = h.y & 0xffffu;
    uint32_t why = 0;  // 0 = accept, else stats slot (5: no packet)
    if (!have) why = 5;
    else if (len < 6u) why = 3;
    else if (flag != 0xf1u && flag != 0xf2u) why = 1;  // ugo/conn.go:395
    const uint32_t row = seqid % a.n;
    const uint64_t grp = seqid / a.n;
    if (!why && (grp < a.first_group || grp >= a.first_group + a.groups)) why = 2;
    const bool acc = why == 0;
    // first copy in ring order?  The claim word is loaded before the payload and
    // only waited for at the stores (a duplicate's payload is loaded, then dropped)
    uint32_t claim = static_cast<uint32_t>(i);
    if (acc && a.win) claim = a.win[(grp - a.first_group) * a.n + row];
    uint64_t before = 0;  // presence at call entry: set = an earlier call placed this seqid
    if (acc && chk_prev) before = a.prev[grp - a.first_group];
    const uint32_t L = acc ? min(len - 6u, a.S) : 0u;  // payload bytes kept
    const uint32_t lim = acc ? L + 6u : 0u;            // packet bytes [0, lim) are needed
    u32x4 A[NP];
    uint32_t bx[NP], by[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const uint32_t o = 16u * (32u * q + hl);
      A[q] = o < lim ? ((NT & 1) ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(pk + o)) : ld16(pk + o))
                     : zero;
      bx[q] = by[q] = 0u;
      if (hl == 31u && o + 16u < lim) {
        const u32x4 B = ld16(pk + o + 16u);
        bx[q] = B.x;
        by[q] = B.y;
      }
    }
    if (acc && claim != static_cast<uint32_t>(i)) why = 4;  // a later copy of a claimed seqid
    if (acc && ((before >> row) & 1ull)) why = 4;           // a copy of an earlier call's seqid
    const bool ok = why == 0;
    uint8_t* dst = a.shards + row * a.rstride + (grp - a.first_group) * a.gstride;
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const uint32_t o = 16u * (32u * q + hl);
      const u32x4 Aq = A[q] ^ K[q];  // bytes past lim are masked below
      // converged: neighbour's chunk (packet bytes [o+16, o+32)) by DPP
      uint32_t nx = from_next_lane(Aq.x), ny = from_next_lane(Aq.y);
      if (hl == 31u) {
        nx = bx[q] ^ kbx[q];
        ny = by[q] ^ kby[q];
      }
      if (!ok || o >= a.S) continue;
      uint32_t w[4];
      if constexpr (MODE == 2) {
        w[0] = Aq.x; w[1] = Aq.y; w[2] = Aq.z; w[3] = Aq.w;
      } else {
        // payload bytes [o, o+16) = packet bytes [o+6, o+22)
        w[0] = __builtin_amdgcn_alignbyte(Aq.z, Aq.y, 2);
        w[1] = __builtin_amdgcn_alignbyte(Aq.w, Aq.z, 2);
        w[2] = __builtin_amdgcn_alignbyte(nx, Aq.w, 2);
        w[3] = __builtin_amdgcn_alignbyte(ny, nx, 2);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {  // zero bytes past the payload
        const uint32_t b0 = o + 4u * j;
        const uint32_t keep = L >= b0 + 4u ? 4u : (L > b0 ? L - b0 : 0u);
        w[j] &= keep >= 4u ? 0xffffffffu : ((1u << (8u * keep)) - 1u);
      }
      const uint32_t nb = a.S - o;
      if (nb >= 16u) {
        const u32x4 v = {w[0], w[1], w[2], w[3]};
        if constexpr (NT & 2)
          __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst + o));
        else
          *reinterpret_cast<u32x4*>(dst + o) = v;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t lo = 4u * j;
          if (nb >= lo + 4u) {
            *reinterpret_cast<uint32_t*>(dst + o + lo) = w[j];
          } else if (nb > lo) {
            for (uint32_t t = 0; t < nb - lo; ++t) dst[o + lo + t] = static_cast<uint8_t>(w[j] >> (8u * t));
          }
        }
      }
    }
    if (hl == 0) {
      if constexpr (MODE == 0)
        acct.issue(a, bstats, why, grp - a.first_group, row);
      else if (why < 5)
        atomicAdd(&bstats[why], 1u);
    }
  }
  if (hl == 0) acct.settle(a, bstats);
  if (a.parts) {
    __syncthreads();
    if (threadIdx.x < 5) a.parts[blockIdx.x * 5u + threadIdx.x] = bstats[threadIdx.x];
  } else if (a.stats) {
    __syncthreads();
    if (threadIdx.x < 5 && bstats[threadIdx.x]) atomicAdd(&a.stats[threadIdx.x], bstats[threadIdx.x]);
  }
}

// Sums per-block counters into stats (one block).
__global__ __launch_bounds__(256) void k_rx_sum_parts(const uint32_t* parts, uint32_t nparts, uint32_t* stats) {
  __shared__ uint32_t tot[5];
  if (threadIdx.x < 5) tot[threadIdx.x] = 0;
  __syncthreads();
  uint32_t c[5] = {0u, 0u, 0u, 0u, 0u};
  for (uint32_t b = threadIdx.x; b < nparts; b += 256u)
#pragma unroll
    for (int k = 0; k < 5; ++k) c[k] += parts[b * 5u + k];
#pragma unroll
  for (int k = 0; k < 5; ++k)
    if (c[k]) atomicAdd(&tot[k], c[k]);
  __syncthreads();
  if (threadIdx.x < 5 && tot[threadIdx.x]) atomicAdd(&stats[threadIdx.x], tot[threadIdx.x]);
}

// ---------------------------------------------------------------------------
// One 16-B output chunk per thread, full grid (k_rx_chunk).
//
// Thread t owns chunk m = t % nq of packet i = t / nq (nq = ceil(S / 16)
// chunks per row): every load it needs -- the packet's header chunk and
// length (shared by the packet's threads: one line per wave), its own payload
// chunk, the keystream -- depends on t alone, so all are issued at once; the
// neighbour chunk the 6-B realignment needs comes from lane + 1 by DPP (a
// separate load only at a packet's last chunk and in lane 63).  With no
// presence bit set at call entry (a->seen, k_rx_begin) there is no snapshot
// lookup.  The packet's chunk-0 thread ORs its presence bit as soon as the
// header is known (DEDUP 1: with the old mask returned -- a bit already set
// is a second copy in this call and raises a.dup for the gated claim and
// re-place; DEDUP 0, timing only: no return).  Blocks keep no counters: the
// rare bad-flag / out-of-window / too-short packets add to sharded words
// (cnt[k * kRxShards + shard], one 128-B line per shard), and k_rx_count
// counts the pieces placed from the presence bits.  This is the access shape
// of the fastest scatter measured (tools/rxgather.hip P2: one chunk per
// thread, full grid).
constexpr uint32_t kRxShards = 32;
constexpr uint32_t kRxShardStride = 32;  // words: one 128-B line per shard
#ifndef UGO_RX_CHUNK  // 1: the chunk path for rows of packets that fit it; 0: the packet-per-half-wave path
#define UGO_RX_CHUNK 0
#endif
constexpr bool kRxChunk = UGO_RX_CHUNK != 0;

__device__ __forceinline__ uint32_t* rx_cnt(uint32_t* cnt, uint32_t k, uint32_t shard) {
  return cnt + (k * kRxShards + shard) * kRxShardStride;
}

template <int NT = 3, int DEDUP = 1>
__global__ __launch_bounds__(256) void k_rx_chunk(RxArgs a, uint32_t nq, uint32_t* cnt) {
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;  // < 2^31 (rx_chunk_ok)
  const uint32_t lane = threadIdx.x & 63u;
  const bool live = t < a.npk * nq;
  const uint32_t i = live ? t / nq : 0u;
  const uint32_t m = t - i * nq;
  const uint32_t o = 16u * m;
  const uint32_t slot = static_cast<uint32_t>(a.slot);
  const uint8_t* pk = a.wire + uint64_t(i) * a.slot;
  const u32x4 zero = {0u, 0u, 0u, 0u};
  // all loads first: header chunk, length, payload chunk, keystream
  u32x4 h = live ? ld16(pk) : zero;
  const uint32_t len = live ? min(static_cast<uint32_t>(a.lens[i]), slot) : 0u;
  u32x4 A = (live && o + 16u <= slot) ? ((NT & 1) ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(pk + o))
                                                  : ld16(pk + o))
                                      : zero;
  const bool own_b = lane == 63u || m + 1u == nq;  // the neighbour chunk is not in lane + 1
  u32x4 B = zero;
  if (live && own_b && o + 32u <= slot) B = ld16(pk + o + 16u);
  if (a.pad) {
    h ^= ld16(a.pad);
    if (o + 16u <= slot) A ^= ld16(a.pad + o);
    if (own_b && o + 32u <= slot) B ^= ld16(a.pad + o + 16u);
  }
  const bool chk_prev = a.prev && !(a.seen && *a.seen < a.call);
  uint32_t why = live ? 0u : 5u;
  const uint32_t seqid = h.x;
  const uint32_t flag = h.y & 0xffffu;
  if (why == 0 && len < 6u) why = 3;
  else if (why == 0 && flag != 0xf1u && flag != 0xf2u) why = 1;  // ugo/conn.go:395
  const uint32_t row = seqid % a.n;
  const uint64_t grp = seqid / a.n;
  if (why == 0 && (grp < a.first_group || grp >= a.first_group + a.groups)) why = 2;
  const uint64_t gs = grp - a.first_group;
  if (why == 0 && chk_prev && ((a.prev[gs] >> row) & 1ull)) why = 4;  // an earlier call's seqid
  [[maybe_unused]] unsigned long long old = 0;
  if constexpr (DEDUP)  // issued now, waited for only at the end
    if (m == 0 && why == 0) old = atomicOr(reinterpret_cast<unsigned long long*>(&a.present[gs]), 1ull << row);
  // neighbour chunk (packet bytes [o+16, o+32)) from lane + 1, converged
  const uint32_t nx = from_next_lane(A.x), ny = from_next_lane(A.y);
  const uint32_t bx = own_b ? B.x : nx, by = own_b ? B.y : ny;
  if (why == 0 && o < a.S) {
    const uint32_t L = min(len - 6u, a.S);  // payload bytes kept
    uint32_t w[4];
    w[0] = __builtin_amdgcn_alignbyte(A.z, A.y, 2);
    w[1] = __builtin_amdgcn_alignbyte(A.w, A.z, 2);
    w[2] = __builtin_amdgcn_alignbyte(bx, A.w, 2);
    w[3] = __builtin_amdgcn_alignbyte(by, bx, 2);
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // zero bytes past the payload
      const uint32_t b0 = o + 4u * j;
      const uint32_t keep = L >= b0 + 4u ? 4u : (L > b0 ? L - b0 : 0u);
      w[j] &= keep >= 4u ? 0xffffffffu : ((1u << (8u * keep)) - 1u);
    }
    uint8_t* dst = a.shards + row * a.rstride + gs * a.gstride + o;
    const uint32_t nb = a.S - o;
    if (nb >= 16u) {
      const u32x4 v = {w[0], w[1], w[2], w[3]};
      if constexpr (NT & 2)
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst));
      else
        *reinterpret_cast<u32x4*>(dst) = v;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t lo = 4u * j;
        if (nb >= lo + 4u) {
          *reinterpret_cast<uint32_t*>(dst + lo) = w[j];
        } else if (nb > lo) {
          for (uint32_t q = 0; q < nb - lo; ++q) dst[lo + q] = static_cast<uint8_t>(w[j] >> (8u * q));
        }
      }
    }
  }
  if (m == 0 && live && why >= 1 && why <= 3 && cnt) atomicAdd(rx_cnt(cnt, why, blockIdx.x % kRxShards), 1u);
  if (m == 0 && why == 0) {
    if constexpr (DEDUP) {
      if ((old >> row) & 1ull) *a.dup = 1u;  // a second copy of this seqid in the call
    } else {
      atomicOr(reinterpret_cast<unsigned long long*>(&a.present[gs]), 1ull << row);
    }
  }
}

// ---------------------------------------------------------------------------
// Destination-ordered RX (index + gather).
//
// k_rx_place writes each packet where its seqid says, in ring order: a block's
// stores are 1470-B pieces scattered over the 13 planar row streams, and the
// 128-B lines where two pieces meet are written half by one block and half by
// another, often on another XCD.  The two kernels below turn that around:
//  1. k_rx_index reads only the 8 header bytes and the length of each packet,
//     classifies it exactly as input does (ugo/fec.go:123-175; conn.go:395)
//     and takes, per (row, group), the smallest packet index (atomicMin: the
//     first copy in ring order wins, ugo/fec.go:123-129).  A (row, group) whose
//     presence bit is already set belongs to an earlier call (duplicate).  The
//     table is row-major -- win[row * groups + g] -- like the planar batch.
//     The atomicMin that finds the word still empty is the one claim that
//     counts as accepted; every other valid packet is a duplicate.  Each block
//     writes its five counters to its own slot of `parts` (no contended
//     device atomics: 2,048 blocks adding into one word cost ~25 us).
//  2. k_rx_gather walks the DESTINATION in order: a full grid, block b owns a
//     contiguous run of (row, group) pieces and writes whole runs of
//     consecutive groups of one row (ORDER 0: the planar rows themselves;
//     ORDER 1: tiles of GT groups, all rows of a tile), reading each piece's
//     packet by the index.  Presence bits are OR-ed per placed piece (no
//     return value, distinct words); block 0 also sums the index kernel's
//     per-block counters into `stats`.
__device__ __forceinline__ uint32_t rx_why(const RxArgs& a, uint32_t len, uint2 hw, uint32_t k0, uint32_t k1,
                                           uint32_t& row, uint64_t& gs) {
  row = 0;
  gs = 0;
  if (len < 6u) return 3;
  const uint32_t seqid = hw.x ^ k0;
  const uint32_t flag = (hw.y ^ k1) & 0xffffu;
  if (flag != 0xf1u && flag != 0xf2u) return 1;  // ugo/conn.go:395
  const uint64_t grp = seqid / a.n;
  if (grp < a.first_group || grp >= a.first_group + a.groups) return 2;
  row = seqid % a.n;
  gs = grp - a.first_group;
  return 0;
}

// PPT packets per thread, all their loads issued first: thread t of block b
// takes packets b*256*PPT + t + 256k.  Per-block counters {accepted, bad flag,
// out of window, too short, duplicate} go to parts[b*5 + k].
template <int PPT>
__global__ __launch_bounds__(256) void k_rx_index(RxArgs a, uint32_t* parts) {
  __shared__ uint32_t bstats[5];
  if (threadIdx.x < 5) bstats[threadIdx.x] = 0;
  __syncthreads();
  uint32_t k0 = 0u, k1 = 0u;
  if (a.pad) {
    k0 = reinterpret_cast<const uint32_t*>(a.pad)[0];
    k1 = reinterpret_cast<const uint32_t*>(a.pad)[1];
  }
  const uint64_t i0 = blockIdx.x * 256ull * PPT + threadIdx.x;
  uint32_t len[PPT];
  uint2 hw[PPT];
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const uint64_t i = i0 + 256u * k;
    len[k] = 0u;
    hw[k] = make_uint2(0u, 0u);
    if (i < a.npk) {
      len[k] = a.lens[i];
      hw[k] = *reinterpret_cast<const uint2*>(a.wire + i * a.slot);
    }
  }
  uint32_t cnt[5] = {0u, 0u, 0u, 0u, 0u};
  uint32_t row[PPT];
  uint64_t gs[PPT];
  bool live[PPT];
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    const uint32_t why = rx_why(a, len[k], hw[k], k0, k1, row[k], gs[k]);
    live[k] = i0 + 256u * k < a.npk && why == 0;
    if (i0 + 256u * k < a.npk && why) ++cnt[why];
  }
  uint64_t pm[PPT];
#pragma unroll
  for (int k = 0; k < PPT; ++k) pm[k] = live[k] ? a.present[gs[k]] : 0ull;
#pragma unroll
  for (int k = 0; k < PPT; ++k) {
    if (!live[k]) continue;
    if ((pm[k] >> row[k]) & 1ull) {  // an earlier call's seqid
      ++cnt[4];
      continue;
    }
    const uint32_t old = atomicMin(&a.win[row[k] * a.groups + gs[k]], static_cast<uint32_t>(i0 + 256u * k));
    ++cnt[old == 0xffffffffu ? 0 : 4];
  }
#pragma unroll
  for (int k = 0; k < 5; ++k)
    if (cnt[k]) atomicAdd(&bstats[k], cnt[k]);
  __syncthreads();
  if (threadIdx.x < 5) parts[blockIdx.x * 5u + threadIdx.x] = bstats[threadIdx.x];
}

// Half a wave per piece (as k_rx_place: 32 lanes x NP passes of 16 B, the
// keystream held in registers, DPP realignment).  The eight half-waves of a
// block take pieces j0 + h, j0 + h + 8, ... of the block's run; the next
// piece's packet index is prefetched one iteration ahead.  NT as k_rx_place.
template <int NP, int ORDER, int GT, int NT = 3>
__global__ __launch_bounds__(256) void k_rx_gather(RxArgs a, const uint32_t* parts, uint32_t nparts) {
  const uint32_t lane = threadIdx.x & 63u, hl = lane & 31u;
  const uint32_t hw = threadIdx.x >> 5;  // half-wave of the block, 0..7
  const u32x4 zero = {0u, 0u, 0u, 0u};
  const uint32_t slot = static_cast<uint32_t>(a.slot);
  if (blockIdx.x == 0 && parts && a.stats) {  // the index kernel's counters
    __shared__ uint32_t tot[5];
    if (threadIdx.x < 5) tot[threadIdx.x] = 0;
    __syncthreads();
    uint32_t c[5] = {0u, 0u, 0u, 0u, 0u};
    for (uint32_t b = threadIdx.x; b < nparts; b += 256u)
#pragma unroll
      for (int k = 0; k < 5; ++k) c[k] += parts[b * 5u + k];
#pragma unroll
    for (int k = 0; k < 5; ++k)
      if (c[k]) atomicAdd(&tot[k], c[k]);
    __syncthreads();
    if (threadIdx.x < 5 && tot[threadIdx.x]) atomicAdd(&a.stats[threadIdx.x], tot[threadIdx.x]);
  }
  const uint64_t ntiles = ORDER == 0 ? a.groups : (a.groups + GT - 1) / GT;
  const uint64_t space = ntiles * (ORDER == 0 ? 1u : GT) * a.n;  // pieces, tail tile included
  const uint64_t unit = ORDER == 0 ? 8u : uint64_t(GT) * a.n;
  uint64_t per = (space + gridDim.x - 1) / gridDim.x;
  per = (per + unit - 1) / unit * unit;
  const uint64_t j0 = blockIdx.x * per;
  const uint64_t j1 = min(space, j0 + per);
  u32x4 K[NP];
  uint32_t kbx[NP], kby[NP];
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const uint32_t o = 16u * (32u * q + hl);
    K[q] = (a.pad && o + 16u <= slot) ? ld16(a.pad + o) : zero;
    kbx[q] = kby[q] = 0u;
    if (a.pad && hl == 31u && o + 32u <= slot) {
      const u32x4 B = ld16(a.pad + o + 16u);
      kbx[q] = B.x;
      kby[q] = B.y;
    }
  }
  auto piece = [&](uint64_t j, uint32_t& row, uint64_t& gs) {
    if constexpr (ORDER == 0) {
      row = static_cast<uint32_t>(j / a.groups);
      gs = j - uint64_t(row) * a.groups;
    } else {
      const uint64_t t = j / (uint64_t(GT) * a.n);
      const uint32_t w = static_cast<uint32_t>(j - t * GT * a.n);
      row = w / GT;
      gs = t * GT + (w - row * GT);
    }
  };
  constexpr uint32_t kNone = 0xffffffffu;
  uint64_t j = j0 + hw;
  uint32_t row_n = 0;
  uint64_t gs_n = 0;
  uint32_t idx_n = kNone;
  if (j < j1) {
    piece(j, row_n, gs_n);
    if (gs_n < a.groups) idx_n = a.win[row_n * a.groups + gs_n];
  }
  for (; j < j1; j += 8) {
    const uint32_t row = row_n, idx = idx_n;
    const uint64_t gs = gs_n;
    if (j + 8 < j1) {  // prefetch the next piece's packet index
      piece(j + 8, row_n, gs_n);
      idx_n = gs_n < a.groups ? a.win[row_n * a.groups + gs_n] : kNone;
    }
    if (idx == kNone) continue;  // half-wave-uniform: lost, or an earlier call's
    const uint8_t* pk = a.wire + uint64_t(idx) * a.slot;
    const uint32_t len = min(static_cast<uint32_t>(a.lens[idx]), slot);  // >= 6: k_rx_index accepted it
    const uint32_t L = min(len - 6u, a.S);
    const uint32_t lim = L + 6u;
    u32x4 A[NP];
    uint32_t bx[NP], by[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const uint32_t o = 16u * (32u * q + hl);
      A[q] = o < lim ? ((NT & 1) ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(pk + o)) : ld16(pk + o))
                     : zero;
      bx[q] = by[q] = 0u;
      if (hl == 31u && o + 16u < lim) {
        const u32x4 B = ld16(pk + o + 16u);
        bx[q] = B.x;
        by[q] = B.y;
      }
    }
    uint8_t* dst = a.shards + row * a.rstride + gs * a.gstride;
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const uint32_t o = 16u * (32u * q + hl);
      const u32x4 Aq = A[q] ^ K[q];
      uint32_t nx = from_next_lane(Aq.x), ny = from_next_lane(Aq.y);
      if (hl == 31u) {
        nx = bx[q] ^ kbx[q];
        ny = by[q] ^ kby[q];
      }
      if (o >= a.S) continue;
      uint32_t w[4];
      w[0] = __builtin_amdgcn_alignbyte(Aq.z, Aq.y, 2);
      w[1] = __builtin_amdgcn_alignbyte(Aq.w, Aq.z, 2);
      w[2] = __builtin_amdgcn_alignbyte(nx, Aq.w, 2);
      w[3] = __builtin_amdgcn_alignbyte(ny, nx, 2);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t b0 = o + 4u * k;
        const uint32_t keep = L >= b0 + 4u ? 4u : (L > b0 ? L - b0 : 0u);
        w[k] &= keep >= 4u ? 0xffffffffu : ((1u << (8u * keep)) - 1u);
      }
      const uint32_t nb = a.S - o;
      if (nb >= 16u) {
        const u32x4 v = {w[0], w[1], w[2], w[3]};
        if constexpr (NT & 2)
          __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst + o));
        else
          *reinterpret_cast<u32x4*>(dst + o) = v;
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t lo = 4u * k;
          if (nb >= lo + 4u) {
            *reinterpret_cast<uint32_t*>(dst + o + lo) = w[k];
          } else if (nb > lo) {
            for (uint32_t t = 0; t < nb - lo; ++t) dst[o + lo + t] = static_cast<uint8_t>(w[k] >> (8u * t));
          }
        }
      }
    }
    if (hl == 0) atomicOr(reinterpret_cast<unsigned long long*>(&a.present[gs]), 1ull << row);
  }
}

// First-arrival claim: one thread per packet reads its 8 header bytes (seqid,
// flag), classifies it exactly as the place kernels do, and takes the
// smallest index per (group, row).  ~8 B read per 1.5-KB packet.
__global__ __launch_bounds__(256) void k_rx_claim(RxArgs a) {
  if (a.cnt) {  // chunk path: gated on k_rx_chunk's duplicate flag; block 0 adds the call's stats
    const bool twice = *a.gate != 0u;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      uint32_t sums[5] = {0u, 0u, 0u, 0u, 0u};
      for (uint32_t k = 1; k < 5; ++k)
        for (uint32_t sh = 0; sh < kRxShards; ++sh) sums[k] += *rx_cnt(a.cnt, k, sh);
      if (a.stats) {  // accepted = pieces placed; duplicates = valid packets not placed
        const uint32_t placed = sums[4], bad = sums[1], oow = sums[2], shrt = sums[3];
        atomicAdd(&a.stats[0], placed);
        if (bad) atomicAdd(&a.stats[1], bad);
        if (oow) atomicAdd(&a.stats[2], oow);
        if (shrt) atomicAdd(&a.stats[3], shrt);
        const uint32_t dups = static_cast<uint32_t>(a.npk) - placed - bad - oow - shrt;
        if (dups) atomicAdd(&a.stats[4], dups);
      }
    }
    if (!twice) return;
  } else if (rx_gated_off(a)) {
    return;
  }
  const uint64_t nthreads = gridDim.x * 256ull;
  uint32_t k0 = 0u, k1 = 0u;
  if (a.pad) {
    k0 = reinterpret_cast<const uint32_t*>(a.pad)[0];
    k1 = reinterpret_cast<const uint32_t*>(a.pad)[1];
  }
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < a.npk; i += nthreads) {
    const uint32_t len = a.lens[i];
    if (len < 6u) continue;
    const uint32_t* h = reinterpret_cast<const uint32_t*>(a.wire + i * a.slot);
    const uint32_t seqid = h[0] ^ k0;
    const uint32_t flag = (h[1] ^ k1) & 0xffffu;
    if (flag != 0xf1u && flag != 0xf2u) continue;
    const uint64_t grp = seqid / a.n;
    if (grp < a.first_group || grp >= a.first_group + a.groups) continue;
    const uint32_t row = seqid % a.n;
    if (a.prev && ((a.prev[grp - a.first_group] >> row) & 1ull)) continue;  // an earlier call's seqid
    atomicMin(&a.win[(grp - a.first_group) * a.n + row], static_cast<uint32_t>(i));
  }
}

__global__ __launch_bounds__(256) void k_rx_fill(uint32_t* win, uint64_t words, const uint32_t* gate) {
  if (gate && *gate == 0u) return;
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < words; i += gridDim.x * 256ull) win[i] = 0xffffffffu;
}

__global__ __launch_bounds__(256) void k_rx_begin(const uint64_t* present, uint64_t* prev, uint64_t groups,
                                                  uint32_t* dup, uint32_t* win, uint64_t words,
                                                  unsigned long long* seen, unsigned long long call, uint32_t* cnt) {
  const uint64_t t = blockIdx.x * 256ull + threadIdx.x;
  const uint64_t nt = gridDim.x * 256ull;
  if (t == 0) *dup = 0u;
  if (cnt)
    for (uint64_t i = t; i < kRxCntWords; i += nt) cnt[i] = 0u;
  uint64_t any = 0;
  for (uint64_t g = t; g < groups; g += nt) {
    const uint64_t m = present[g];
    prev[g] = m;
    any |= m;
  }
  if (win)
    for (uint64_t i = t; i < words; i += nt) win[i] = 0xffffffffu;
  if (seen && __any(any != 0) && (threadIdx.x & 63u) == 0) atomicMax(seen, call);
}

hipError_t launch_rx_begin(const uint64_t* present, uint64_t* prev, uint64_t groups, uint32_t* dup, uint32_t* win,
                           uint64_t words, unsigned long long* seen, unsigned long long call, hipStream_t s,
                           uint32_t* cnt) {
  uint64_t blocks = (groups + 255) / 256;
  if (blocks == 0) blocks = 1;
  if (blocks > 1024u) blocks = 1024u;
  launch(kKRx, k_rx_begin, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s, present, prev, groups, dup, win,
         words, seen, call, cnt);
  return hipGetLastError();
}

// Per group, the presence bits this call set (present & ~prev): their sum is
// the number of (group, row) pieces the call placed.  Sharded adds, one per block.
__global__ __launch_bounds__(256) void k_rx_count(const uint64_t* present, const uint64_t* prev, uint64_t groups,
                                                  uint32_t* cnt) {
  __shared__ uint32_t tot;
  if (threadIdx.x == 0) tot = 0;
  __syncthreads();
  uint32_t c = 0;
  for (uint64_t g = blockIdx.x * 256ull + threadIdx.x; g < groups; g += gridDim.x * 256ull)
    c += __popcll(present[g] & ~prev[g]);
  if (c) atomicAdd(&tot, c);
  __syncthreads();
  if (threadIdx.x == 0 && tot) atomicAdd(rx_cnt(cnt, 4, blockIdx.x % kRxShards), tot);
}

hipError_t launch_rx_count(const RxArgs& a, hipStream_t s) {
  uint64_t blocks = (a.groups + 255) / 256;
  if (blocks == 0) blocks = 1;
  if (blocks > 64u) blocks = 64u;
  launch(kKRx, k_rx_count, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s, a.present, a.prev, a.groups, a.cnt);
  return hipGetLastError();
}

bool rx_chunk_ok(const RxArgs& a) {
  const uint64_t nq = (a.S + 15u) / 16u;
  // a packet's chunks must cover its payload: nq chunks of packet bytes [16m, 16m + 16) for m < nq,
  // plus the neighbour (realignment) -- within the slot
  return kRxChunk && nq >= 1 && a.npk * nq < (1ull << 31) && 16u * nq <= a.slot;
}

hipError_t launch_rx_chunk(const RxArgs& a, hipStream_t s) {
  const uint32_t nq = (a.S + 15u) / 16u;
  const uint64_t items = a.npk * nq;
  if (items == 0) return hipSuccess;
  launch(kKRx, k_rx_chunk<3>, dim3(static_cast<uint32_t>((items + 255) / 256)), dim3(256), 0, s, a, nq, a.cnt);
  return hipGetLastError();
}

hipError_t launch_rx_fill(uint32_t* win, uint64_t words, const uint32_t* gate, hipStream_t s) {
  uint64_t blocks = (words + 255) / 256;
  if (blocks == 0) return hipSuccess;
  if (blocks > 1024u) blocks = 1024u;
  launch(kKRx, k_rx_fill, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s, win, words, gate);
  return hipGetLastError();
}

static inline uint32_t rx_blocks(const RxArgs& a) {
  const uint64_t waves = (a.npk + 1) / 2;
  uint64_t blocks = (waves + 3) / 4;
  if (blocks > 2048u) blocks = 2048u;  // 8 workgroups per CU, grid-stride over packet pairs
  return static_cast<uint32_t>(blocks);
}

hipError_t launch_rx_claim(const RxArgs& a, hipStream_t s) {
  uint64_t blocks = (a.npk + 255) / 256;
  if (blocks == 0) return hipSuccess;
  if (blocks > 4096u) blocks = 4096u;
  launch(kKRx, k_rx_claim, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_rx_scatter(const RxArgs& a, hipStream_t s) {
  const uint32_t blocks = rx_blocks(a);
  if (blocks == 0) return hipSuccess;
  const uint32_t passes = ((a.S + 15u) / 16u + 31u) / 32u;
  // nt loads + stores: on a cold ring and batch 493 vs 552 us with plain ones
  // (a linear copy of the same bytes: 487 us; tools/rxvariants 15 cold)
  switch (passes) {
    case 1: launch(kKRx, k_rx_place<1, 0, 3>, dim3(blocks), dim3(256), 0, s, a); break;
    case 2: launch(kKRx, k_rx_place<2, 0, 3>, dim3(blocks), dim3(256), 0, s, a); break;
    case 3: launch(kKRx, k_rx_place<3, 0, 3>, dim3(blocks), dim3(256), 0, s, a); break;
    case 4: launch(kKRx, k_rx_place<4, 0, 3>, dim3(blocks), dim3(256), 0, s, a); break;
    default: launch(kKRx, k_rx_scatter, dim3(blocks), dim3(256), 0, s, a); break;
  }
  return hipGetLastError();
}

}  // namespace kern
}  // namespace ugo
