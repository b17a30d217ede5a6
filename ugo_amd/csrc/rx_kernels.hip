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

// 16 bytes at any byte address (one global_load_dwordx4: gfx950 runs with
// unaligned access enabled)
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
template <bool NTL>
__device__ __forceinline__ u32x4 ldu16(const uint8_t* p) {
  if constexpr (NTL)
    return __builtin_nontemporal_load(reinterpret_cast<const u32x4u*>(p));
  else
    return *reinterpret_cast<const u32x4u*>(p);
}

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

// Realigns, masks and stores one output chunk of a packet: payload bytes
// [o, o + 16) = packet bytes [o + 6, o + 22) = bytes 6..15 of the lane's chunk
// A and bytes 0..5 of the next one (nx, ny); bytes at or past the kept length
// L (<= S) are zero.  Always a whole 16-B chunk: a row's last chunk carries
// zeros past S up to round_up(S, 16) (include/ugo_fec.h).  Writing only the
// row's S bytes left every row's last 64-B line partially written, and that
// cost 6 % of the RX call's time in order, 3 % shuffled (466.9 vs 494.9 us,
// 499.1 vs 512.4; tools/rxgather.hip, profiles/r5/rxgather/r5_rxtail4_*) --
// while one unaligned 16-B store of the row's last 16 payload bytes, which
// leaves the padding unwritten, gained nothing (498.2 / 529.3 us): the partial
// line, not the store count, is the cost.
// TAILB (round 5): the byte masks only for a chunk that reaches past L, behind
// a branch -- a packet has one such chunk, in one of its passes, so a wave
// skips the masks in the passes where none of its lanes holds one: VALU
// instructions 128.5 -> 94.0 per packet, time unchanged (454.9 vs 454.7 us in
// order, 468.4 vs 468.3 shuffled; profiles/r5/rxpmc/, rxgather/r5_tailb.jsonl):
// the kernel is not VALU-bound.  TAILB 0: masks on every chunk (A/B).
template <int NTS, int TAILB = 1>
__device__ __forceinline__ void rx_put(uint8_t* row, uint32_t o, uint32_t L, const u32x4& A, uint32_t nx,
                                       uint32_t ny) {
  uint32_t w[4];
  w[0] = __builtin_amdgcn_alignbyte(A.z, A.y, 2);
  w[1] = __builtin_amdgcn_alignbyte(A.w, A.z, 2);
  w[2] = __builtin_amdgcn_alignbyte(nx, A.w, 2);
  w[3] = __builtin_amdgcn_alignbyte(ny, nx, 2);
  if (!TAILB || o + 16u > L) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // zero bytes past the payload
      const uint32_t b0 = o + 4u * j;
      const uint32_t keep = L >= b0 + 4u ? 4u : (L > b0 ? L - b0 : 0u);
      w[j] &= keep >= 4u ? 0xffffffffu : ((1u << (8u * keep)) - 1u);
    }
  }
  const u32x4 v = {w[0], w[1], w[2], w[3]};
  if constexpr (NTS)
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(row + o));
  else
    *reinterpret_cast<u32x4*>(row + o) = v;
}

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
      if (ok && o < a.S) rx_put<0>(dst, o, L, A, bx, by);  // whole chunks (rx_put)
    }
    if (hl == 0) acct.issue(a, bstats, why, gs, row);
  }
  if (hl == 0) acct.settle(a, bstats);
  if (a.stats) {
    __syncthreads();
    if (threadIdx.x < 5 && bstats[threadIdx.x]) atomicAdd(&a.stats[threadIdx.x], bstats[threadIdx.x]);
  }
}

// The loads-first place kernel (its A/B forms: tools/rx_experiments.hpp
// k_rx_place) with the header taken from the payload's own first chunk: lane 0
// of a half loads packet bytes [0, 16) as part of the payload anyway, so the
// header and flag come to the other lanes by ds_bpermute instead of a separate
// (prefetched) header load: one memory instruction less per packet pair
// (468.6 / 489.8 vs 476.4 / 494.9 us, profiles/r4/rxgather_hdr_*).  Loading
// the lengths 32 iterations at a time as well gains nothing measurable
// (rxgather_lenbatch_*).  Production.
// Every lane loads the bytes [0, min(len, S + 6)) of its packet before the
// header is known (a packet later rejected for its flag or window is loaded
// and dropped, like a duplicate).  Realignment as MODE 4.
// RUNS (A/B): 0 = grid-stride over packet pairs (wave w: pairs w, w + nwaves,
// ...); 1 = each wave takes one contiguous run of packet pairs, so the line a
// packet's slot shares with the next packet's is read by the same wave.
template <int NP, int NT = 3, int RUNS = 0, int TAILB = 1>
__global__ __launch_bounds__(256) void k_rx_place_h(RxArgs a) {
  if (rx_gated_off(a)) return;
  __shared__ uint32_t bstats[5];
  if (threadIdx.x < 5) bstats[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, half = lane >> 5, hl = lane & 31u;
  const uint64_t wave = (blockIdx.x * 256ull + threadIdx.x) >> 6;
  const uint64_t nwaves = (gridDim.x * 256ull) >> 6;
  const u32x4 zero = {0u, 0u, 0u, 0u};
  const uint32_t slot = static_cast<uint32_t>(a.slot);
  const bool chk_prev = a.prev && !(a.seen && *a.seen < a.call);
  u32x4 K[NP];
  uint32_t kbx = 0u, kby = 0u;  // keystream of lane 31's last-pass neighbour chunk
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const uint32_t o = 16u * (32u * q + hl);
    K[q] = (a.pad && o + 16u <= slot) ? ld16(a.pad + o) : zero;
    if (q == NP - 1 && a.pad && hl == 31u && o + 32u <= slot) {
      const u32x4 B = ld16(a.pad + o + 16u);
      kbx = B.x;
      kby = B.y;
    }
  }
  RxAccount acct;
  uint64_t first = 2 * wave, step = 2 * nwaves, end = a.npk;
  if constexpr (RUNS) {  // wave w: packets [w * run, (w + 1) * run), run even
    const uint64_t run = ((a.npk + nwaves - 1) / nwaves + 1) & ~1ull;
    first = wave * run;
    step = 2;
    end = min(a.npk, first + run);
  }
  const int hsrc = static_cast<int>(half * 32u) * 4;  // lane 0 of this half
  uint64_t i = first + half;
  uint32_t ln = i < end ? a.lens[i] : 0u;
  for (uint64_t base = first; base < end; base += step, i += step) {
    const bool have = i < end;
    const uint8_t* pk = a.wire + i * a.slot;
    const uint32_t len = have ? min(ln, slot) : 0u;
    if (i + step < end) ln = a.lens[i + step];  // the next packet's length
    const uint32_t lim = len >= 6u ? min(len, a.S + 6u) : 0u;  // packet bytes [0, lim) may be kept
    u32x4 A[NP];
    uint32_t bx = 0u, by = 0u;
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const uint32_t o = 16u * (32u * q + hl);
      A[q] = o < lim ? ((NT & 1) ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(pk + o)) : ld16(pk + o))
                     : zero;
      if (q == NP - 1 && hl == 31u && o + 16u < lim) {
        const u32x4 B = ld16(pk + o + 16u);
        bx = B.x;
        by = B.y;
      }
    }
    const u32x4 A0 = A[0] ^ K[0];  // lane 0: packet bytes [0, 16) = the header
    const uint32_t seqid = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(hsrc, static_cast<int>(A0.x)));
    const uint32_t flag = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(hsrc, static_cast<int>(A0.y))) & 0xffffu;
    uint32_t why = 0;  // 0 = accept, else stats slot (5: no packet)
    if (!have) why = 5;
    else if (len < 6u) why = 3;
    else if (flag != 0xf1u && flag != 0xf2u) why = 1;  // ugo/conn.go:395
    const uint32_t row = seqid % a.n;
    const uint64_t grp = seqid / a.n;
    if (!why && (grp < a.first_group || grp >= a.first_group + a.groups)) why = 2;
    const bool acc = why == 0;
    uint32_t claim = static_cast<uint32_t>(i);
    if (acc && a.win) claim = a.win[(grp - a.first_group) * a.n + row];
    uint64_t before = 0;
    if (acc && chk_prev) before = a.prev[grp - a.first_group];
    const uint32_t L = acc ? min(len - 6u, a.S) : 0u;  // payload bytes kept
    if (acc && claim != static_cast<uint32_t>(i)) why = 4;  // a later copy of a claimed seqid
    if (acc && ((before >> row) & 1ull)) why = 4;           // a copy of an earlier call's seqid
    const bool ok = why == 0;
    uint8_t* dst = a.shards + row * a.rstride + (grp - a.first_group) * a.gstride;
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const uint32_t o = 16u * (32u * q + hl);
      const u32x4 Aq = A[q] ^ K[q];
      uint32_t nx, ny;
      if (q + 1 < NP) {  // lane l takes lane l+1's chunk, lane 31 lane 0's next-pass chunk
        const u32x4 An = A[q + 1 < NP ? q + 1 : q] ^ K[q + 1 < NP ? q + 1 : q];
        const uint32_t sx = hl == 0u ? An.x : Aq.x, sy = hl == 0u ? An.y : Aq.y;
        const int src = static_cast<int>(hl == 31u ? lane - 31u : lane + 1u) * 4;
        nx = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(sx)));
        ny = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(sy)));
      } else {
        nx = from_next_lane(Aq.x);
        ny = from_next_lane(Aq.y);
        if (hl == 31u) {
          nx = bx ^ kbx;
          ny = by ^ kby;
        }
      }
      if (!ok || o >= a.S) continue;
      rx_put<(NT & 2), TAILB>(dst, o, L, Aq, nx, ny);
    }
    if (hl == 0) acct.issue(a, bstats, why, grp - a.first_group, row);
  }
  if (hl == 0) acct.settle(a, bstats);
  if (a.stats) {
    __syncthreads();
    if (threadIdx.x < 5 && bstats[threadIdx.x]) atomicAdd(&a.stats[threadIdx.x], bstats[threadIdx.x]);
  }
}

// Frame rows (ugo_fec_rx_assemble_frames, round 6): row seqid % n of a group
// receives the decrypted packet itself -- bytes [0, min(len, S + 6)), zeros up
// to round_up(S + 6, 16) -- so the payload sits at column 6 of the row.  A
// packet chunk lands at the same offset it was loaded from: no realignment, so
// none of the place kernel's per-chunk neighbour exchange (two ds_bpermute per
// chunk, lane 31's extra load, the funnel shift of rx_put).  GF columns are
// independent, so Reconstruct over the frame window (shard size S + 6) gives
// the payload columns bit for bit; the 6 header columns of a recovered row are
// a combination of the survivors' headers and are ignored.  This is the frame
// TX already keeps (k_tx_c: a lane holds packet bytes [16m, 16m + 16)).
// Presence, first-copy rule, stats and gated passes as k_rx_place_h.
// Measured (round 6, tools/rx_frames_ab.py, one box, same storage): 2.4-4 %
// under the uncapped payload kernel; against the payload kernel capped as this
// one, a tie (4 bench runs: -4.0 / -4.0 / +1.3 / +2.8 % in order, within 0.6 %
// shuffled; profiles/r6/rx_frames/final_tree_runs.json); residency 3 blocks/CU (0.512 vs 0.539-0.553 ms at
// 5 or uncapped, pitch 1488); rows at a 64-B pitch written to whole lines
// (1536 for S = 1470: 0.40-0.46 vs 0.51-0.55 ms at the 1488 pitch); the same
// frames one chunk per thread over the whole ring (the P2 shape, every lane
// loading its packet's header and length) 0.58-0.63 ms -- a dependent header
// load per lane outweighs the cheaper store pattern
// (profiles/r6/rx_frames/p2_one_chunk_per_thread_ab.jsonl).
__device__ __forceinline__ u32x4 rx_keep(u32x4 v, uint32_t o, uint32_t lim) {
  // bytes at or past lim of the chunk at o become zero (only a packet's tail chunk)
  if (o + 16u <= lim) return v;
  const uint32_t keep = lim > o ? lim - o : 0u;
  uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t b0 = 4u * j;
    const uint32_t k = keep >= b0 + 4u ? 4u : (keep > b0 ? keep - b0 : 0u);
    w[j] &= k >= 4u ? 0xffffffffu : ((1u << (8u * k)) - 1u);
  }
  return u32x4{w[0], w[1], w[2], w[3]};
}

template <int NP>
__global__ __launch_bounds__(256) void k_rx_frame_h(RxArgs a) {
  if (rx_gated_off(a)) return;
  __shared__ uint32_t bstats[5];
  if (threadIdx.x < 5) bstats[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, half = lane >> 5, hl = lane & 31u;
  const uint64_t wave = (blockIdx.x * 256ull + threadIdx.x) >> 6;
  const uint64_t nwaves = (gridDim.x * 256ull) >> 6;
  const u32x4 zero = {0u, 0u, 0u, 0u};
  const uint32_t slot = static_cast<uint32_t>(a.slot);
  const uint32_t FS = a.S + 6u;  // frame bytes kept per row
  const uint32_t FW = a.fill;     // bytes written per row (zeros past FS)
  const bool chk_prev = a.prev && !(a.seen && *a.seen < a.call);
  u32x4 K[NP];
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const uint32_t o = 16u * (32u * q + hl);
    K[q] = (a.pad && o + 16u <= slot) ? ld16(a.pad + o) : zero;
  }
  RxAccount acct;
  const uint64_t step = 2 * nwaves;
  const int hsrc = static_cast<int>(half * 32u) * 4;  // lane 0 of this half
  uint64_t i = 2 * wave + half;
  uint32_t ln = i < a.npk ? a.lens[i] : 0u;
  for (uint64_t base = 2 * wave; base < a.npk; base += step, i += step) {
    const bool have = i < a.npk;
    const uint8_t* pk = a.wire + i * a.slot;
    const uint32_t len = have ? min(ln, slot) : 0u;
    if (i + step < a.npk) ln = a.lens[i + step];  // the next packet's length
    const uint32_t lim = len >= 6u ? min(len, FS) : 0u;  // packet bytes [0, lim) are kept
    u32x4 A[NP];
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const uint32_t o = 16u * (32u * q + hl);
      A[q] = o < lim ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(pk + o)) : zero;
    }
    const u32x4 A0 = A[0] ^ K[0];  // lane 0: packet bytes [0, 16) = the header
    const uint32_t seqid = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(hsrc, static_cast<int>(A0.x)));
    const uint32_t flag = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(hsrc, static_cast<int>(A0.y))) & 0xffffu;
    uint32_t why = 0;
    if (!have) why = 5;
    else if (len < 6u) why = 3;
    else if (flag != 0xf1u && flag != 0xf2u) why = 1;  // ugo/conn.go:395
    const uint32_t row = seqid % a.n;
    const uint64_t grp = seqid / a.n;
    if (!why && (grp < a.first_group || grp >= a.first_group + a.groups)) why = 2;
    const bool acc = why == 0;
    uint32_t claim = static_cast<uint32_t>(i);
    if (acc && a.win) claim = a.win[(grp - a.first_group) * a.n + row];
    uint64_t before = 0;
    if (acc && chk_prev) before = a.prev[grp - a.first_group];
    if (acc && claim != static_cast<uint32_t>(i)) why = 4;
    if (acc && ((before >> row) & 1ull)) why = 4;
    const bool ok = why == 0;
    uint8_t* dst = a.shards + row * a.rstride + (grp - a.first_group) * a.gstride;
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const uint32_t o = 16u * (32u * q + hl);
      if (!ok || o >= FW) continue;
      __builtin_nontemporal_store(rx_keep(A[q] ^ K[q], o, lim), reinterpret_cast<u32x4*>(dst + o));
    }
    if (hl == 0) acct.issue(a, bstats, why, grp - a.first_group, row);
  }
  if (hl == 0) acct.settle(a, bstats);
  if (a.stats) {
    __syncthreads();
    if (threadIdx.x < 5 && bstats[threadIdx.x]) atomicAdd(&a.stats[threadIdx.x], bstats[threadIdx.x]);
  }
}

// Frame rows wider than 4 passes of 32 chunks (S + 6 > 2048, e.g. jumbo
// packets): the same placement in a loop over passes, the header loaded by
// every lane of the half (one broadcast request).
__global__ __launch_bounds__(256) void k_rx_frame_scatter(RxArgs a) {
  if (rx_gated_off(a)) return;
  __shared__ uint32_t bstats[5];
  if (threadIdx.x < 5) bstats[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, half = lane >> 5, hl = lane & 31u;
  const uint64_t wave = (blockIdx.x * 256ull + threadIdx.x) >> 6;
  const uint64_t nwaves = (gridDim.x * 256ull) >> 6;
  const uint32_t slot = static_cast<uint32_t>(a.slot);
  const uint32_t FS = a.S + 6u;
  const uint32_t nq = a.fill / 16u;
  const u32x4 zero = {0u, 0u, 0u, 0u};
  const u32x4 K0 = a.pad ? ld16(a.pad) : zero;
  RxAccount acct;
  const uint64_t step = 2 * nwaves;
  uint64_t i = 2 * wave + half;
  for (uint64_t base = 2 * wave; base < a.npk; base += step, i += step) {
    const bool have = i < a.npk;
    const uint8_t* pk = a.wire + i * a.slot;
    const uint32_t len = have ? min(static_cast<uint32_t>(a.lens[i]), slot) : 0u;
    const uint32_t lim = len >= 6u ? min(len, FS) : 0u;
    u32x4 h = zero;
    if (lim) h = ld16(pk) ^ K0;
    const uint32_t seqid = h.x;
    const uint32_t flag = h.y & 0xffffu;
    uint32_t why = 0;
    if (!have) why = 5;
    else if (len < 6u) why = 3;
    else if (flag != 0xf1u && flag != 0xf2u) why = 1;  // ugo/conn.go:395
    const uint32_t row = seqid % a.n;
    const uint64_t grp = seqid / a.n;
    if (!why && (grp < a.first_group || grp >= a.first_group + a.groups)) why = 2;
    const uint64_t gs = grp - a.first_group;
    if (!why && a.prev && ((a.prev[gs] >> row) & 1ull)) why = 4;
    if (!why && a.win && a.win[gs * a.n + row] != static_cast<uint32_t>(i)) why = 4;
    if (why == 0) {
      uint8_t* dst = a.shards + row * a.rstride + gs * a.gstride;
      for (uint32_t q = hl; q < nq; q += 32u) {
        const uint32_t o = 16u * q;
        u32x4 v = zero;
        if (o < lim) {
          v = ld16(pk + o);
          if (a.pad && o + 16u <= slot) v ^= ld16(a.pad + o);
        }
        *reinterpret_cast<u32x4*>(dst + o) = rx_keep(v, o, lim);
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

// First-arrival claim: one thread per packet reads its 8 header bytes (seqid,
// flag), classifies it exactly as the place kernels do, and takes the
// smallest index per (group, row).  ~8 B read per 1.5-KB packet.
__global__ __launch_bounds__(256) void k_rx_claim(RxArgs a) {
  if (rx_gated_off(a)) return;
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
                                                  unsigned long long* seen, unsigned long long call) {
  const uint64_t t = blockIdx.x * 256ull + threadIdx.x;
  const uint64_t nt = gridDim.x * 256ull;
  if (t == 0) *dup = 0u;
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

// Frame rows -> payload rows: out row r = bytes [off, off + S) of src row r,
// zeros to round_up(S, 16); one thread per 16-B output chunk (two aligned
// source chunks, funnel shift).  The host RX path's recovered rows on their
// way out (only those rows: ~4 % of a ring's bytes), so the D2H copy reads
// 16-B aligned rows.
__global__ __launch_bounds__(256) void k_shift_rows(const uint8_t* src, uint64_t spitch, uint32_t off, uint8_t* dst,
                                                    uint64_t dpitch, uint32_t S, uint64_t rows) {
  const uint32_t nq = (S + 15u) / 16u;
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i >= rows * nq) return;
  const uint64_t r = i / nq;
  const uint32_t q = static_cast<uint32_t>(i - r * nq);
  const uint32_t o = 16u * q + off;      // first source byte of this chunk
  const uint32_t a0 = o & ~15u, sh = o & 15u;
  const uint8_t* row = src + r * spitch;
  const u32x4 A = ld16(row + a0);
  u32x4 B = {0u, 0u, 0u, 0u};
  if (sh && a0 + 16u < off + S) B = ld16(row + a0 + 16u);  // the next chunk holds bytes of this one
  const uint32_t w8[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
  uint32_t w[4];
  const uint32_t dw = sh >> 2, bs = sh & 3u;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    uint32_t lo = 0u, hi = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k)  // select without runtime-indexed arrays (dw < 4)
      if (dw == static_cast<uint32_t>(k)) {
        lo = w8[j + k];
        hi = w8[j + k + 1 < 8 ? j + k + 1 : 7];
      }
    w[j] = __builtin_amdgcn_alignbyte(hi, lo, bs);
  }
  const uint32_t L = S - 16u * q;  // payload bytes of this chunk (zeros past S)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t b0 = 4u * j;
    const uint32_t k = L >= b0 + 4u ? 4u : (L > b0 ? L - b0 : 0u);
    w[j] &= k >= 4u ? 0xffffffffu : ((1u << (8u * k)) - 1u);
  }
  *reinterpret_cast<u32x4*>(dst + r * dpitch + 16u * q) = u32x4{w[0], w[1], w[2], w[3]};
}

hipError_t launch_shift_rows(const uint8_t* src, uint64_t spitch, uint32_t off, uint8_t* dst, uint64_t dpitch,
                             uint32_t S, uint64_t rows, hipStream_t s) {
  const uint64_t items = rows * ((S + 15u) / 16u);
  if (items == 0) return hipSuccess;
  launch(kKRx, k_shift_rows, dim3(static_cast<uint32_t>((items + 255) / 256)), dim3(256), 0, s, src, spitch, off, dst,
         dpitch, S, rows);
  return hipGetLastError();
}

hipError_t launch_rx_begin(const uint64_t* present, uint64_t* prev, uint64_t groups, uint32_t* dup, uint32_t* win,
                           uint64_t words, unsigned long long* seen, unsigned long long call, hipStream_t s) {
  uint64_t blocks = (groups + 255) / 256;
  if (blocks == 0) blocks = 1;
  if (blocks > 1024u) blocks = 1024u;
  launch(kKRx, k_rx_begin, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s, present, prev, groups, dup, win,
         words, seen, call);
  return hipGetLastError();
}

hipError_t launch_rx_fill(uint32_t* win, uint64_t words, const uint32_t* gate, hipStream_t s) {
  uint64_t blocks = (words + 255) / 256;
  if (blocks == 0) return hipSuccess;
  if (blocks > 1024u) blocks = 1024u;
  launch(kKRx, k_rx_fill, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s, win, words, gate);
  return hipGetLastError();
}

#ifndef UGO_RX_GRID_BLOCKS
#define UGO_RX_GRID_BLOCKS 16384u
#endif
static inline uint32_t rx_blocks(const RxArgs& a) {
  const uint64_t waves = (a.npk + 1) / 2;
  uint64_t blocks = (waves + 3) / 4;
  // grid-stride over packet pairs; 16384 blocks (~6 packets per half-wave on
  // the bench ring, each keeping its keystream chunks in registers): with
  // k_rx_place_h 0.3-1.5% faster than 8192 on two boxes and 2.5% faster than
  // 4096, 32768 no better (profiles/r4/rxgather_hgrid_*.jsonl, _g16k_*; _grid_*
  // for the earlier form)
  if (blocks > UGO_RX_GRID_BLOCKS) blocks = UGO_RX_GRID_BLOCKS;
  return static_cast<uint32_t>(blocks);
}

// A gated pass (a.gate set) mostly finds its gate closed -- no duplicate in
// the call -- and then costs its grid's dispatch: 1024 grid-stride blocks
// instead of a full grid take 4 us off the call (profiles/r5/rxgather/
// r5_gated_*; with duplicates the re-place is ~10% slower on the smaller grid).
#ifndef UGO_RX_GATED_BLOCKS
#define UGO_RX_GATED_BLOCKS 1024
#endif
constexpr uint64_t kRxGatedBlocks = UGO_RX_GATED_BLOCKS;

hipError_t launch_rx_claim(const RxArgs& a, hipStream_t s) {
  uint64_t blocks = (a.npk + 255) / 256;
  if (blocks == 0) return hipSuccess;
  if (blocks > kRxGatedBlocks) blocks = kRxGatedBlocks;
  launch(kKRx, k_rx_claim, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s, a);
  return hipGetLastError();
}

// Residency cap of the frame kernels: dynamic LDS they never touch holds them
// to kRxFrameBlocks blocks per CU (0: none, the VGPR-limited occupancy).
#ifndef UGO_RX_FRAME_BLOCKS
#define UGO_RX_FRAME_BLOCKS 3
#endif
static uint32_t rx_frame_lds() {
  static const uint32_t cap = [] {
    if (UGO_RX_FRAME_BLOCKS <= 0) return 0u;
    int dev = 0, lds = 160 * 1024;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess ||
        lds <= 4096)
      lds = 160 * 1024;
    return static_cast<uint32_t>(lds / UGO_RX_FRAME_BLOCKS - 1024);
  }();
  return cap;
}

// Residency cap of the payload place kernel too (round 6): 3 blocks per CU
// by unused LDS, as the frame kernel -- against its VGPR-limited 5 waves per
// SIMD the payload rows' gap to frame rows on the same storage shrank from
// 1.1-1.7 % to 0.3-0.8 % in order (4 blocks: 0.8-1.0 %), one box, three
// allocations (profiles/r6/rx_frames/place_cap_ab.jsonl).  0: no cap.
#ifndef UGO_RX_PLACE_BLOCKS
#define UGO_RX_PLACE_BLOCKS 3
#endif
static uint32_t rx_place_lds() {
  static const uint32_t cap = [] {
    if (UGO_RX_PLACE_BLOCKS <= 0) return 0u;
    int dev = 0, lds = 160 * 1024;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess ||
        lds <= 4096)
      lds = 160 * 1024;
    return static_cast<uint32_t>(lds / UGO_RX_PLACE_BLOCKS - 1024);
  }();
  return cap;
}

hipError_t launch_rx_scatter(const RxArgs& a, hipStream_t s) {
  uint32_t blocks = rx_blocks(a);
  if (a.gate && blocks > kRxGatedBlocks) blocks = static_cast<uint32_t>(kRxGatedBlocks);
  if (blocks == 0) return hipSuccess;
  if (a.frame) {  // frame rows: no realignment (k_rx_frame_h)
    const uint32_t lds = rx_frame_lds();
    switch ((a.fill / 16u + 31u) / 32u) {
      case 1: launch(kKRx, k_rx_frame_h<1>, dim3(blocks), dim3(256), lds, s, a); break;
      case 2: launch(kKRx, k_rx_frame_h<2>, dim3(blocks), dim3(256), lds, s, a); break;
      case 3: launch(kKRx, k_rx_frame_h<3>, dim3(blocks), dim3(256), lds, s, a); break;
      case 4: launch(kKRx, k_rx_frame_h<4>, dim3(blocks), dim3(256), lds, s, a); break;
      default: launch(kKRx, k_rx_frame_scatter, dim3(blocks), dim3(256), lds, s, a); break;
    }
    return hipGetLastError();
  }
  const uint32_t passes = ((a.S + 15u) / 16u + 31u) / 32u;
  // nt loads + stores: on a cold ring and batch 493 vs 552 us with plain ones
  // (a linear copy of the same bytes: 487 us; tools/rxvariants 15 cold)
  // the header from the payload's first chunk, the realignment's neighbour
  // chunks by ds_bpermute: no header or neighbour loads
  const uint32_t plds = rx_place_lds();
  switch (passes) {
    case 1: launch(kKRx, k_rx_place_h<1, 3>, dim3(blocks), dim3(256), plds, s, a); break;
    case 2: launch(kKRx, k_rx_place_h<2, 3>, dim3(blocks), dim3(256), plds, s, a); break;
    case 3: launch(kKRx, k_rx_place_h<3, 3>, dim3(blocks), dim3(256), plds, s, a); break;
    case 4: launch(kKRx, k_rx_place_h<4, 3>, dim3(blocks), dim3(256), plds, s, a); break;
    default: launch(kKRx, k_rx_scatter, dim3(blocks), dim3(256), 0, s, a); break;
  }
  return hipGetLastError();
}

}  // namespace kern
}  // namespace ugo
