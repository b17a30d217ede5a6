// rx_experiments.hpp -- RX assembly kernels measured in round 4 and not
// shipped (tools/rxgather.hip times them against production; results in
// profiles/r4/rxgather_*.jsonl).  Included after
// ugo_amd/csrc/rx_kernels.hip, whose helpers (ld16, from_next_lane, RxArgs,
// launch_rx_claim) they use.  Not product code.
//
//  * chunk path: k_rx_chunk (one 16-B output chunk per thread, full grid) +
//    k_rx_count + k_rx_chunk_stats, 597-600 us against production's 523-535 us;
//  * production's place kernel over a full grid + k_rx_tally_full: 712-722 us
//    against 500-518 (every packet reloads its lane's keystream chunks);
//  * destination-ordered index + gather (k_rx_index, k_rx_gather), slower still.
#pragma once

namespace ugo {
namespace kern {

// Loads-first form for rows of at most 32 * NP chunks (NP = 3 for ugo's
// 1470-B payloads).  Same decomposition (half a wave per packet), but:
//  * the keystream chunks at a lane's offsets are the same for every packet,
//    so they are loaded once and held in registers;
//  * the next packet's header and length are prefetched, so a packet's
//    placement is known before its payload arrives, and all NP payload loads of
//    a packet are issued before its first store (the per-pass load -> store
//    chain of k_rx_scatter kept one 1-KiB load in flight per wave);
//  * lengths are clamped to the slot.
// (Production is k_rx_place_h in ugo_amd/csrc/rx_kernels.hip.)  MODE: 4 = aligned loads realigned with the right neighbour's
// chunk, which lane l of a half takes from lane l+1 and lane 31 from lane 0's
// next-pass chunk, all by one ds_bpermute (no neighbour loads; 492.7 / 490.5
// vs 504.3 / 499.1 us in order / shuffled, profiles/r4/rxgather_bperm_*);
// 0 = the round-3 form (DPP from lane l+1, lane 31 loads its neighbour).  A/B
// only (tools/rxgather.hip, profiles/r4/rxgather_{attribution,unaligned}_*):
// 1 = MODE 0 without the presence atomics (timing only, -5 us), 2 = the same
// loads and stores without the realignment (timing only, -20 us), 3 =
// unaligned payload loads instead of the realignment (bit-exact, +13 us).
// NT: bit 0 nontemporal payload loads, bit 1 nontemporal stores.
// RARE (A/B only, tools/rx_experiments.hpp full-grid path): 1 = a block adds
// only its bad-flag / out-of-window / too-short counts to a.stats (the call's
// scratch counters; accepted and duplicates are tallied from the presence bits
// afterwards).  The full grid lost: 712 vs 500 us.
template <int NP, int MODE = 0, int NT = 0, int RARE = 0>
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
    kbx[q] = kby[q] = 0u;
    if constexpr (MODE == 3) {  // keystream at the payload's offsets, unaligned
      K[q] = (a.pad && o + 22u <= slot) ? ldu16<false>(a.pad + 6u + o) : zero;
      continue;
    }
    K[q] = (a.pad && o + 16u <= slot) ? ld16(a.pad + o) : zero;
    if (a.pad && hl == 31u && o + 32u <= slot) {
      const u32x4 B = ld16(a.pad + o + 16u);
      kbx[q] = B.x;
      kby[q] = B.y;
    }
  }
  RxAccount acct;
  // grid-stride over packet pairs
  const uint64_t first = 2 * wave, step = 2 * nwaves, end = a.npk;
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
      bx[q] = by[q] = 0u;
      if constexpr (MODE == 3) {  // payload bytes [o, o+16) directly (host: 16*floor((S-1)/16) + 22 <= slot)
        A[q] = o < L ? ldu16<(NT & 1) != 0>(pk + 6u + o) : zero;
        continue;
      }
      A[q] = o < lim ? ((NT & 1) ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(pk + o)) : ld16(pk + o))
                     : zero;
      if (MODE == 4 && q + 1 < NP) continue;  // lane 31's neighbour is lane 0's next chunk
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
      uint32_t nx = 0u, ny = 0u;
      if constexpr (MODE == 4) {
        if (q + 1 < NP) {
          // lane l of a half takes lane l+1's chunk; lane 31 takes lane 0's
          // chunk of the next pass (packet bytes [o+16, o+32)), which lane 0
          // sends instead of its own: no neighbour load
          const u32x4 An = A[q + 1 < NP ? q + 1 : q] ^ K[q + 1 < NP ? q + 1 : q];
          const uint32_t sx = hl == 0u ? An.x : Aq.x, sy = hl == 0u ? An.y : Aq.y;
          const int src = static_cast<int>(hl == 31u ? lane - 31u : lane + 1u) * 4;
          nx = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(sx)));
          ny = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(sy)));
        } else {
          nx = from_next_lane(Aq.x);
          ny = from_next_lane(Aq.y);
          if (hl == 31u) {
            nx = bx[q] ^ kbx[q];
            ny = by[q] ^ kby[q];
          }
        }
      } else if constexpr (MODE != 3) {
        nx = from_next_lane(Aq.x);
        ny = from_next_lane(Aq.y);
        if (hl == 31u) {
          nx = bx[q] ^ kbx[q];
          ny = by[q] ^ kby[q];
        }
      }
      if (!ok || o >= a.S) continue;
      uint32_t w[4];
      if constexpr (MODE == 2 || MODE == 3) {
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
      if constexpr (MODE == 0 || MODE == 3 || MODE == 4)
        acct.issue(a, bstats, why, grp - a.first_group, row);
      else if (why < 5)
        atomicAdd(&bstats[why], 1u);
    }
  }
  if (hl == 0) acct.settle(a, bstats);
  if (a.stats) {
    __syncthreads();
    const bool mine = RARE ? (threadIdx.x >= 1 && threadIdx.x <= 3) : threadIdx.x < 5;
    if (mine && bstats[threadIdx.x]) atomicAdd(&a.stats[threadIdx.x], bstats[threadIdx.x]);
  }
}


// Chunk-path counters: (-, bad flag, out of window, too short, pieces placed)
// x 32 shards, one 128-B line per shard (32 shards on one line serialized the
// adds: 1740 us).
constexpr uint32_t kRxShards = 32;
constexpr uint32_t kRxShardStride = 32;  // words
constexpr uint32_t kRxCntWords = 5 * kRxShards * kRxShardStride;

__device__ __forceinline__ uint32_t* rx_cnt(uint32_t* cnt, uint32_t k, uint32_t shard) {
  return cnt + (k * kRxShards + shard) * kRxShardStride;
}

__global__ __launch_bounds__(256) void k_rx_zero_cnt(uint32_t* cnt) {
  for (uint32_t i = threadIdx.x; i < kRxCntWords; i += 256u) cnt[i] = 0u;
}

// Thread t owns chunk m = t % nq of packet i = t / nq (nq = ceil(S / 16)):
// every load it needs -- the packet's header chunk and length, its payload
// chunk, the keystream -- depends on t alone, so all are issued at once; the
// neighbour chunk of the 6-B realignment comes from lane + 1 by DPP.  The
// packet's chunk-0 thread ORs its presence bit (DEDUP 1: with the old mask
// returned -- a bit already set is a second copy in this call and raises
// a.dup; DEDUP 0, timing only: no return).  Rare classes add to sharded words.
template <int NT = 3, int DEDUP = 1>
__global__ __launch_bounds__(256) void k_rx_chunk(RxArgs a, uint32_t nq, uint32_t* cnt) {
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;  // < 2^31 (caller's check)
  const uint32_t lane = threadIdx.x & 63u;
  const bool live = t < a.npk * nq;
  const uint32_t i = live ? t / nq : 0u;
  const uint32_t m = t - i * nq;
  const uint32_t o = 16u * m;
  const uint32_t slot = static_cast<uint32_t>(a.slot);
  const uint8_t* pk = a.wire + uint64_t(i) * a.slot;
  const u32x4 zero = {0u, 0u, 0u, 0u};
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
  if constexpr (DEDUP)
    if (m == 0 && why == 0) old = atomicOr(reinterpret_cast<unsigned long long*>(&a.present[gs]), 1ull << row);
  const uint32_t nx = from_next_lane(A.x), ny = from_next_lane(A.y);
  const uint32_t bx = own_b ? B.x : nx, by = own_b ? B.y : ny;
  if (why == 0 && o < a.S) {
    const uint32_t L = min(len - 6u, a.S);
    uint32_t w[4];
    w[0] = __builtin_amdgcn_alignbyte(A.z, A.y, 2);
    w[1] = __builtin_amdgcn_alignbyte(A.w, A.z, 2);
    w[2] = __builtin_amdgcn_alignbyte(bx, A.w, 2);
    w[3] = __builtin_amdgcn_alignbyte(by, bx, 2);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
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
      if ((old >> row) & 1ull) *a.dup = 1u;
    } else {
      atomicOr(reinterpret_cast<unsigned long long*>(&a.present[gs]), 1ull << row);
    }
  }
}

// Per group, the presence bits this call set (present & ~prev): their sum is
// the number of (group, row) pieces the call placed.
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

// The call's stats from the sharded counters (one thread), for the chunk path;
// the claim itself is production's k_rx_claim, gated on the dup flag.
__global__ void k_rx_chunk_stats(const uint32_t* cnt, uint32_t* stats, uint64_t npk) {
  uint32_t sums[5] = {0u, 0u, 0u, 0u, 0u};
  for (uint32_t k = 1; k < 5; ++k)
    for (uint32_t sh = 0; sh < kRxShards; ++sh) sums[k] += cnt[(k * kRxShards + sh) * kRxShardStride];
  const uint32_t placed = sums[4], bad = sums[1], oow = sums[2], shrt = sums[3];
  stats[0] += placed;
  stats[1] += bad;
  stats[2] += oow;
  stats[3] += shrt;
  stats[4] += static_cast<uint32_t>(npk) - placed - bad - oow - shrt;
}

// The chunk path as ugo_fec_rx_assemble ran it under UGO_RX_CHUNK (round 4):
// begin -> zero counters -> chunk -> count -> stats -> gated claim -> gated re-place.
inline hipError_t launch_rx_chunk_path(RxArgs a, uint64_t* prev, uint32_t* win, uint32_t* dup, uint32_t* cnt,
                                       unsigned long long* seen, unsigned long long call, hipStream_t s) {
  hipError_t e = launch_rx_begin(a.present, prev, a.groups, dup, win, a.groups * a.n, seen, call, s);
  if (e != hipSuccess) return e;
  k_rx_zero_cnt<<<1, 256, 0, s>>>(cnt);
  a.seen = seen;
  a.call = call;
  a.dup = dup;
  a.prev = prev;
  RxArgs f = a;
  f.win = win;
  f.gate = dup;
  f.dup = nullptr;
  f.stats = nullptr;
  f.fixup = 1;
  const uint32_t nq = (a.S + 15u) / 16u;
  const uint64_t items = a.npk * nq;
  if (items) k_rx_chunk<3><<<static_cast<uint32_t>((items + 255) / 256), 256, 0, s>>>(a, nq, cnt);
  uint64_t blocks = (a.groups + 255) / 256;
  if (blocks > 64u) blocks = 64u;
  k_rx_count<<<static_cast<uint32_t>(blocks ? blocks : 1), 256, 0, s>>>(a.present, prev, a.groups, cnt);
  if (a.stats) k_rx_chunk_stats<<<1, 1, 0, s>>>(cnt, a.stats, a.npk);
  e = launch_rx_claim(f, s);
  if (e != hipSuccess) return e;
  return launch_rx_scatter(f, s);
}

// ---------------------------------------------------------------------------
// Full-grid place: k_rx_place with one packet per half-wave (blocks =
// ceil(npk / 8), the P3b shape) -- per-block stats adds would contend, so the
// blocks add only the rare classes to the call's scratch counters rare[1..3]
// (RARE = 1) and k_rx_tally_full turns the presence bits this call set into the
// accepted count: stats[0] += placed, stats[1..3] += rare[1..3],
// stats[4] += npk - placed - rare (every other valid packet was a duplicate).
// Each block adds its share of placed (wrapping uint32 arithmetic).
__global__ __launch_bounds__(256) void k_rx_tally_full(const uint64_t* present, const uint64_t* prev, uint64_t groups,
                                                  const uint32_t* rare, uint32_t* stats, uint64_t npk) {
  __shared__ uint32_t tot;
  if (threadIdx.x == 0) tot = 0;
  __syncthreads();
  uint32_t c = 0;
  for (uint64_t g = blockIdx.x * 256ull + threadIdx.x; g < groups; g += gridDim.x * 256ull)
    c += __popcll(present[g] & ~prev[g]);
  if (c) atomicAdd(&tot, c);
  __syncthreads();
  if (threadIdx.x == 0) {
    if (tot) {
      atomicAdd(&stats[0], tot);
      atomicSub(&stats[4], tot);
    }
    if (blockIdx.x == 0) {
      const uint32_t r1 = rare[1], r2 = rare[2], r3 = rare[3];
      if (r1) atomicAdd(&stats[1], r1);
      if (r2) atomicAdd(&stats[2], r2);
      if (r3) atomicAdd(&stats[3], r3);
      atomicAdd(&stats[4], static_cast<uint32_t>(npk) - r1 - r2 - r3);
    }
  }
}

__global__ void k_rx_zero_rare(uint32_t* rare) {
  if (threadIdx.x < 8) rare[threadIdx.x] = 0u;
}

// begin -> zero rare -> full-grid place (RARE) -> tally -> gated claim -> gated re-place (grid-stride)
inline hipError_t launch_rx_full_path(RxArgs a, uint64_t* prev, uint32_t* win, uint32_t* dup, uint32_t* rare,
                                      unsigned long long* seen, unsigned long long call, hipStream_t s) {
  hipError_t e = launch_rx_begin(a.present, prev, a.groups, dup, win, a.groups * a.n, seen, call, s);
  if (e != hipSuccess) return e;
  k_rx_zero_rare<<<1, 64, 0, s>>>(rare);
  a.seen = seen;
  a.call = call;
  a.dup = dup;
  a.prev = prev;
  RxArgs f = a;
  f.win = win;
  f.gate = dup;
  f.dup = nullptr;
  f.stats = nullptr;
  f.fixup = 1;
  uint32_t* user_stats = a.stats;
  a.stats = user_stats ? rare : nullptr;
  const uint32_t blocks = static_cast<uint32_t>((a.npk + 7) / 8);
  if (blocks) k_rx_place<3, 0, 3, 1><<<blocks, 256, 0, s>>>(a);
  if (user_stats) {
    uint64_t tb = (a.groups + 255) / 256;
    if (tb > 64u) tb = 64u;
    k_rx_tally_full<<<static_cast<uint32_t>(tb ? tb : 1), 256, 0, s>>>(a.present, prev, a.groups, rare, user_stats,
                                                               a.npk);
  }
  e = launch_rx_claim(f, s);
  if (e != hipSuccess) return e;
  return launch_rx_scatter(f, s);
}

// ---------------------------------------------------------------------------
// Destination-ordered RX (index + gather).  k_rx_index reads only the header
// and length of each packet, classifies it and takes the smallest packet index
// per (row, group) (atomicMin; row-major table win[row * groups + g]); each
// block writes its five counters to parts[b*5 + k].  k_rx_gather walks the
// destination in order (ORDER 0: planar rows; ORDER 1: tiles of GT groups),
// half a wave per piece.
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
    if ((pm[k] >> row[k]) & 1ull) {
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

template <int NP, int ORDER, int GT, int NT = 3>
__global__ __launch_bounds__(256) void k_rx_gather(RxArgs a, const uint32_t* parts, uint32_t nparts) {
  const uint32_t lane = threadIdx.x & 63u, hl = lane & 31u;
  const uint32_t hw = threadIdx.x >> 5;
  const u32x4 zero = {0u, 0u, 0u, 0u};
  const uint32_t slot = static_cast<uint32_t>(a.slot);
  if (blockIdx.x == 0 && parts && a.stats) {
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
  const uint64_t space = ntiles * (ORDER == 0 ? 1u : GT) * a.n;
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
    if (j + 8 < j1) {
      piece(j + 8, row_n, gs_n);
      idx_n = gs_n < a.groups ? a.win[row_n * a.groups + gs_n] : kNone;
    }
    if (idx == kNone) continue;
    const uint8_t* pk = a.wire + uint64_t(idx) * a.slot;
    const uint32_t len = min(static_cast<uint32_t>(a.lens[idx]), slot);
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


// ---------------------------------------------------------------------------
// Round-5 full-grid forms (tools/rxgather.hip).  Both take the
// call's 8 control words `ctl` (zeroed by k_rx_zero_rare before the kernel):
// [0] duplicate gate, [1] pieces placed, [2..5] packets of the rare classes 1..4,
// [6] k_rx_tally's block count.  Results (profiles/r5/rxgather_*): k_rx_slots
// 540-630 us against production's 489-499 (its block barriers cost more than
// the one global load per lane they save); k_rx_half ties production (486.5 /
// 516.4 vs 489.0 / 512.9), and with whole-chunk row tails 458.7 / 499.0 vs
// production's 466.9 / 499.1 -- but it reads whole slots whatever the packet
// length, so a ring of short packets would read many times its bytes;
// production keeps the length-aware loads.
// ---------------------------------------------------------------------------
// Slot-linear placement (round 5).  Thread t of a block owns slot chunk
// m = t % T of packet i = P * blockIdx.x + t / T (T = slot / 16 chunks, or
// ceil(S / 16) if that is more): the block's P * T threads read P whole slots
// exactly as a plain nt copy reads them -- consecutive lanes on consecutive
// 16-B chunks, one chunk per thread, a full grid (the compute-free P2 pattern's
// shape).  What a lane needs from another lane comes through
// LDS, behind two block barriers:
//  * the keystream (PADLDS): staged once per block, P slots' worth of packets
//    per 1.5-KB stage instead of one L2 reload per packet (the cost that sank
//    the round-4 full-grid forms); PADLDS 0 loads it per thread (A/B);
//  * the header: chunk 0's lane decrypts it, classifies the packet, ORs its
//    presence bit and publishes (group, row, kept length);
//  * the realignment's right neighbour: the first 8 B of chunk m + 1.
// No per-packet counter atomics: a block adds only its rare classes to the
// call's control words, and k_rx_tally derives the accepted count from the
// presence bits the call set (present & ~prev) -- and raises the duplicate
// gate when accepted + rare falls short of the packet count, i.e. when two
// copies of one seqid were both placed (the gated claim / re-place passes then
// keep the first copy, as for k_rx_place_h).
struct RxHdr {
  uint64_t gs;   // group in the batch
  uint32_t row;  // seqid % n
  uint32_t L;    // payload bytes kept; kRxSkip: the packet writes nothing
};
constexpr uint32_t kRxSkip = 0xffffffffu;

template <int PADLDS>
__global__ __launch_bounds__(1024) void k_rx_slots(RxArgs a, uint32_t T, uint32_t P, uint32_t* ctl) {
  extern __shared__ __attribute__((aligned(16))) uint8_t rx_smem[];
  __shared__ uint32_t scnt[5];
  const uint32_t slot = static_cast<uint32_t>(a.slot);
  const uint32_t Q = slot / 16u;  // chunks per slot (<= T)
  u32x4* spad = reinterpret_cast<u32x4*>(rx_smem);                             // [Q] (PADLDS)
  RxHdr* shdr = reinterpret_cast<RxHdr*>(rx_smem + (PADLDS ? 16u * Q : 0u));  // [P]
  uint2* snb = reinterpret_cast<uint2*>(shdr + P);                             // [P * T]
  const uint32_t t = threadIdx.x;
  const uint32_t lp = t / T, m = t - lp * T;
  const uint64_t i = uint64_t(blockIdx.x) * P + lp;
  const bool live = i < a.npk;
  const u32x4 zero = {0u, 0u, 0u, 0u};
  const uint8_t* pk = a.wire + i * a.slot;
  u32x4 K = zero;
  if constexpr (PADLDS) {
    if (a.pad)
      for (uint32_t q = t; q < Q; q += blockDim.x) spad[q] = ld16(a.pad + 16u * q);
  } else {
    if (a.pad && m < Q) K = ld16(a.pad + 16u * m);
  }
  u32x4 A = zero;
  if (live && m < Q) A = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(pk + 16u * m));
  uint32_t len = 0u;
  if (live && m == 0u) len = min(static_cast<uint32_t>(a.lens[i]), slot);
  if (t < 5u) scnt[t] = 0u;
  const bool chk_prev = a.prev && !(a.seen && *a.seen < a.call);
  __syncthreads();
  if constexpr (PADLDS) {
    if (a.pad && m < Q) K = spad[m];
  }
  A ^= K;
  snb[t] = make_uint2(A.x, A.y);
  if (live && m == 0u) {  // packet bytes [0, 16): the FEC header (ugo/fec.go:78-89)
    const uint32_t seqid = A.x, flag = A.y & 0xffffu;
    uint32_t why = 0;
    if (len < 6u) why = 3;
    else if (flag != 0xf1u && flag != 0xf2u) why = 1;  // ugo/conn.go:395
    const uint32_t row = seqid % a.n;
    const uint64_t grp = seqid / a.n;
    if (!why && (grp < a.first_group || grp >= a.first_group + a.groups)) why = 2;
    const uint64_t gs = grp - a.first_group;
    if (!why && chk_prev && ((a.prev[gs] >> row) & 1ull)) why = 4;  // an earlier call placed this seqid
    RxHdr h;
    h.gs = gs;
    h.row = row;
    h.L = why ? kRxSkip : min(len - 6u, a.S);  // copy(buf, data[6:]) bounded by the row
    shdr[lp] = h;
    if (why == 0)
      atomicOr(reinterpret_cast<unsigned long long*>(&a.present[gs]), 1ull << row);
    else
      atomicAdd(&scnt[why], 1u);
  }
  __syncthreads();
  if (t >= 1u && t <= 4u && scnt[t]) atomicAdd(&ctl[1 + t], scnt[t]);
  if (!live) return;
  const RxHdr h = shdr[lp];
  const uint32_t o = 16u * m;  // payload bytes [o, o+16) = packet bytes [o+6, o+22)
  if (h.L == kRxSkip || o >= a.S) return;
  const uint2 nb = m + 1u < Q ? snb[t + 1u] : make_uint2(0u, 0u);
  uint32_t w[4];
  w[0] = __builtin_amdgcn_alignbyte(A.z, A.y, 2);
  w[1] = __builtin_amdgcn_alignbyte(A.w, A.z, 2);
  w[2] = __builtin_amdgcn_alignbyte(nb.x, A.w, 2);
  w[3] = __builtin_amdgcn_alignbyte(nb.y, nb.x, 2);
  const uint32_t L = h.L;
#pragma unroll
  for (int j = 0; j < 4; ++j) {  // zero bytes past the payload
    const uint32_t b0 = o + 4u * j;
    const uint32_t keep = L >= b0 + 4u ? 4u : (L > b0 ? L - b0 : 0u);
    w[j] &= keep >= 4u ? 0xffffffffu : ((1u << (8u * keep)) - 1u);
  }
  uint8_t* dst = a.shards + h.row * a.rstride + h.gs * a.gstride + o;
  const uint32_t nbytes = a.S - o;
  if (nbytes >= 16u) {
    __builtin_nontemporal_store(u32x4{w[0], w[1], w[2], w[3]}, reinterpret_cast<u32x4*>(dst));
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t lo = 4u * j;
      if (nbytes >= lo + 4u) {
        *reinterpret_cast<uint32_t*>(dst + lo) = w[j];
      } else if (nbytes > lo) {
        for (uint32_t q = 0; q < nbytes - lo; ++q) dst[lo + q] = static_cast<uint8_t>(w[j] >> (8u * q));
      }
    }
  }
}

// Full-grid half-wave placement (round 5, the P3b shape): half a wave per
// packet, 8 packets per 256-thread block, one packet pair per wave, no loop.
// Unlike k_rx_place_h every load a lane issues is independent of every other
// load: the payload chunks are read whole slot (no length-dependent predicate),
// the length and the keystream (PADMODE 0: per lane from L1/L2; 1: staged once
// per block in LDS) alongside, so a wave has one memory round trip before its
// stores, not a length -> payload -> header chain.  Stats and the duplicate
// gate as k_rx_slots (ctl + k_rx_tally); the presence atomicOr returns nothing.
// ATTR (A/B attribution only, tools/rxgather.hip; 0 in production): 1 no
// keystream, 2 no presence atomic, 4 whole 16-B store of the tail chunk (writes
// the row's padding), 8 no length load, 16 no realignment.
template <int NP, int PADMODE, int ATTR = 0, int LNT = 1>
__global__ __launch_bounds__(256) void k_rx_half(RxArgs a, uint32_t* ctl) {
  __shared__ u32x4 spad[PADMODE ? 32 * NP + 1 : 1];
  const uint32_t lane = threadIdx.x & 63u, half = lane >> 5, hl = lane & 31u;
  const uint64_t i = blockIdx.x * 8ull + (threadIdx.x >> 5);
  const bool live = i < a.npk;
  const uint32_t slot = static_cast<uint32_t>(a.slot);
  const uint32_t Q = slot / 16u;
  const u32x4 zero = {0u, 0u, 0u, 0u};
  const uint8_t* pk = a.wire + i * a.slot;
  u32x4 K[NP], A[NP];
  if constexpr (PADMODE) {
    if (a.pad)
      for (uint32_t q = threadIdx.x; q < Q; q += 256u) spad[q] = ld16(a.pad + 16u * q);
  } else {
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const uint32_t m = 32u * q + hl;
      K[q] = (!(ATTR & 1) && a.pad && m < Q) ? ld16(a.pad + 16u * m) : zero;
    }
  }
  const uint32_t len = live ? ((ATTR & 8) ? slot - 12u : min(static_cast<uint32_t>(a.lens[i]), slot)) : 0u;
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const uint32_t m = 32u * q + hl;
    A[q] = (live && m < Q) ? (LNT ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(pk + 16u * m))
                                  : ld16(pk + 16u * m))
                           : zero;
  }
  const bool chk_prev = a.prev && !(a.seen && *a.seen < a.call);
  if constexpr (PADMODE) {
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NP; ++q) {
      const uint32_t m = 32u * q + hl;
      K[q] = (a.pad && m < Q) ? spad[m] : zero;
    }
  }
#pragma unroll
  for (int q = 0; q < NP; ++q) A[q] ^= K[q];
  const int hsrc = static_cast<int>(half * 32u) * 4;  // lane 0 of this half: packet bytes [0, 16)
  const uint32_t seqid = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(hsrc, static_cast<int>(A[0].x)));
  const uint32_t flag = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(hsrc, static_cast<int>(A[0].y))) & 0xffffu;
  uint32_t why = 0;
  if (!live) why = 5;
  else if (len < 6u) why = 3;
  else if (flag != 0xf1u && flag != 0xf2u) why = 1;  // ugo/conn.go:395
  const uint32_t row = seqid % a.n;
  const uint64_t grp = seqid / a.n;
  if (!why && (grp < a.first_group || grp >= a.first_group + a.groups)) why = 2;
  const uint64_t gs = grp - a.first_group;
  if (!why && chk_prev && ((a.prev[gs] >> row) & 1ull)) why = 4;  // an earlier call placed this seqid
  if (hl == 0u) {
    if (why == 0 && !(ATTR & 2))
      atomicOr(reinterpret_cast<unsigned long long*>(&a.present[gs]), 1ull << row);
    else if (why < 5)
      atomicAdd(&ctl[1 + why], 1u);
  }
  const uint32_t L = why == 0 ? min(len - 6u, a.S) : 0u;
  uint8_t* dst = a.shards + row * a.rstride + gs * a.gstride;
#pragma unroll
  for (int q = 0; q < NP; ++q) {
    const uint32_t o = 16u * (32u * q + hl);
    uint32_t nx, ny;
    if (q + 1 < NP) {  // lane l takes lane l+1's chunk, lane 31 lane 0's next-pass chunk
      const u32x4 An = A[q + 1 < NP ? q + 1 : q];
      const uint32_t sx = hl == 0u ? An.x : A[q].x, sy = hl == 0u ? An.y : A[q].y;
      const int src = static_cast<int>(hl == 31u ? lane - 31u : lane + 1u) * 4;
      nx = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(sx)));
      ny = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src, static_cast<int>(sy)));
    } else {  // lane 31's neighbour, chunk 32 * NP, lies past the slot
      nx = from_next_lane(A[q].x);
      ny = from_next_lane(A[q].y);
      if (hl == 31u) nx = ny = 0u;
    }
    if (why != 0 || o >= a.S) continue;
    if constexpr (ATTR & 20) {  // attribution forms (timing only)
      uint32_t w[4];
      if constexpr (ATTR & 16) {
        w[0] = A[q].x; w[1] = A[q].y; w[2] = A[q].z; w[3] = A[q].w;
      } else {
        w[0] = __builtin_amdgcn_alignbyte(A[q].z, A[q].y, 2);
        w[1] = __builtin_amdgcn_alignbyte(A[q].w, A[q].z, 2);
        w[2] = __builtin_amdgcn_alignbyte(nx, A[q].w, 2);
        w[3] = __builtin_amdgcn_alignbyte(ny, nx, 2);
      }
      __builtin_nontemporal_store(u32x4{w[0], w[1], w[2], w[3]}, reinterpret_cast<u32x4*>(dst + o));
    } else {
      rx_put<1>(dst, o, L, A[q], nx, ny);
    }
  }
}

// After k_rx_slots: pieces placed = popcount(present & ~prev) over the window;
// the last block to finish adds the call's stats and sets the duplicate gate
// ctl[0] when placed + rare < npk (two copies of a seqid were both placed).
__global__ __launch_bounds__(256) void k_rx_tally(const uint64_t* present, const uint64_t* prev, uint64_t groups,
                                                  uint32_t* ctl, uint32_t* stats, uint64_t npk) {
  __shared__ uint32_t tot;
  if (threadIdx.x == 0) tot = 0u;
  __syncthreads();
  uint32_t c = 0u;
  for (uint64_t g = blockIdx.x * 256ull + threadIdx.x; g < groups; g += gridDim.x * 256ull)
    c += static_cast<uint32_t>(__popcll(present[g] & ~prev[g]));
  if (c) atomicAdd(&tot, c);
  __syncthreads();
  if (threadIdx.x != 0) return;
  if (tot) atomicAdd(&ctl[1], tot);
  __threadfence();
  if (atomicAdd(&ctl[6], 1u) != gridDim.x - 1u) return;
  __threadfence();
  const uint32_t placed = atomicAdd(&ctl[1], 0u);
  const uint32_t r1 = atomicAdd(&ctl[2], 0u), r2 = atomicAdd(&ctl[3], 0u), r3 = atomicAdd(&ctl[4], 0u),
                 r4 = atomicAdd(&ctl[5], 0u);
  const uint32_t np = static_cast<uint32_t>(npk);
  if (placed + r1 + r2 + r3 + r4 != np) ctl[0] = 1u;
  if (stats) {
    if (placed) atomicAdd(&stats[0], placed);
    if (r1) atomicAdd(&stats[1], r1);
    if (r2) atomicAdd(&stats[2], r2);
    if (r3) atomicAdd(&stats[3], r3);
    const uint32_t dups = np - placed - r1 - r2 - r3;
    if (dups) atomicAdd(&stats[4], dups);
  }
}



// ---------------------------------------------------------------------------
// k_rx_p2 (round 5): the P2 pattern's shape -- one 16-B slot chunk per lane,
// a full grid, consecutive lanes on consecutive chunks -- with everything
// per-packet done on the scalar unit.  Wave w covers slot chunks [63w, 63w+64)
// of the ring (93 per 1488-B slot): 64 < 93, so the wave touches at most two
// packets, whose headers, lengths, classification and snapshot words it reads
// with scalar loads; lanes 0..62 store an output chunk, lane 63 only lends its
// chunk to lane 62's realignment (DPP), so a wave issues ONE payload load and
// ONE store.  The keystream: per lane from L1/L2 (PADLDS 0) or staged in LDS
// behind one block barrier that the payload loads stay in flight across
// (PADLDS 1).  Presence / rare classes / duplicate gate as k_rx_half (ctl +
// k_rx_tally).  Needs slot >= 1024 B (64 chunks) and S <= slot.
typedef const __attribute__((address_space(4))) uint32_t* rx_cptr;

__device__ __forceinline__ uint32_t rx_sld(const void* p) { return *(rx_cptr)(p); }

struct RxPk {  // one packet's placement, wave-uniform
  uint64_t gs;
  uint32_t row, L, why;
};

__device__ __forceinline__ RxPk rx_classify(const RxArgs& a, uint64_t i, uint32_t k0, uint32_t k1, bool chk_prev) {
  RxPk r{0, 0, 0, 5};
  if (i >= a.npk) return r;
  const uint32_t slot = static_cast<uint32_t>(a.slot);
  const uint8_t* pk = a.wire + i * a.slot;
  const uint32_t seqid = rx_sld(pk) ^ k0;
  const uint32_t flag = (rx_sld(pk + 4) ^ k1) & 0xffffu;
  const uintptr_t la = reinterpret_cast<uintptr_t>(a.lens + i);
  const uint32_t lw = rx_sld(reinterpret_cast<const void*>(la & ~uintptr_t(3)));
  const uint32_t len = min((la & 2) ? (lw >> 16) : (lw & 0xffffu), slot);
  uint32_t why = 0;
  if (len < 6u) why = 3;
  else if (flag != 0xf1u && flag != 0xf2u) why = 1;  // ugo/conn.go:395
  r.row = seqid % a.n;
  const uint64_t grp = seqid / a.n;
  if (!why && (grp < a.first_group || grp >= a.first_group + a.groups)) why = 2;
  r.gs = grp - a.first_group;
  if (!why && chk_prev) {
    const uint32_t* pw = reinterpret_cast<const uint32_t*>(a.prev + r.gs);
    const uint32_t bit = r.row < 32u ? (rx_sld(pw) >> r.row) : (rx_sld(pw + 1) >> (r.row - 32u));
    if (bit & 1u) why = 4;  // an earlier call placed this seqid
  }
  r.why = why;
  r.L = why ? 0u : min(len - 6u, a.S);
  return r;
}

// LEN 1: the lengths of the wave's two packets by scalar loads FIRST, and a
// lane loads its chunk only if it starts inside its packet (length-aware
// loads, as production's, at the price of a scalar round trip before them).
__device__ __forceinline__ uint32_t rx_slen(const RxArgs& a, uint64_t i) {
  if (i >= a.npk) return 0u;
  const uintptr_t la = reinterpret_cast<uintptr_t>(a.lens + i);
  const uint32_t lw = rx_sld(reinterpret_cast<const void*>(la & ~uintptr_t(3)));
  return min((la & 2) ? (lw >> 16) : (lw & 0xffffu), static_cast<uint32_t>(a.slot));
}

template <int PADLDS, int LEN = 0>
__global__ __launch_bounds__(256) void k_rx_p2(RxArgs a, uint32_t* ctl) {
  __shared__ u32x4 spad[PADLDS ? 128 : 1];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t Q = static_cast<uint32_t>(a.slot / 16u);
  const uint64_t w = uint64_t(blockIdx.x) * 4u + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t total = a.npk * Q;
  const uint64_t c0 = 63u * w;  // the wave's first chunk (uniform)
  const uint64_t c = c0 + lane;
  bool live = c < total;
  const uint64_t i = c / Q;
  const uint32_t m = static_cast<uint32_t>(c - i * Q);
  const u32x4 zero = {0u, 0u, 0u, 0u};
  if constexpr (LEN) {  // chunk m is needed only if it starts inside the packet (the left neighbour may need it)
    const uint64_t j0 = c0 / Q;
    const uint32_t l0 = rx_slen(a, j0), l1 = rx_slen(a, j0 + 1);
    const uint32_t lim = min(i != j0 ? l1 : l0, a.S + 6u);
    live = live && 16u * m < lim;
  }
  u32x4 A = live ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.wire + i * a.slot + 16u * m)) : zero;
  u32x4 K = zero;
  if constexpr (PADLDS) {
    if (a.pad)
      for (uint32_t q = threadIdx.x; q < Q; q += 256u) spad[q] = ld16(a.pad + 16u * q);
    __syncthreads();
    if (a.pad && live) K = spad[m];
  } else {
    if (a.pad && live) K = ld16(a.pad + 16u * m);
  }
  if (c0 >= total) return;  // wave-uniform (after the block barrier)
  const uint32_t k0 = a.pad ? rx_sld(a.pad) : 0u, k1 = a.pad ? rx_sld(a.pad + 4) : 0u;
  const bool chk_prev = a.prev && !(a.seen && *a.seen < a.call);
  const uint64_t i0 = c0 / Q;
  const RxPk p0 = rx_classify(a, i0, k0, k1, chk_prev);
  const RxPk p1 = rx_classify(a, i0 + 1, k0, k1, chk_prev);  // the wave's second packet, if it reaches it
  const bool second = i != i0;
  const uint32_t why = second ? p1.why : p0.why;
  const uint32_t row = second ? p1.row : p0.row;
  const uint64_t gs = second ? p1.gs : p0.gs;
  const uint32_t L = second ? p1.L : p0.L;
  // the packet's chunk-0 lane accounts for it -- not lane 63, whose chunk is
  // the next wave's lane 0 (it would count the packet twice)
  if (lane < 63u && c < total && m == 0u) {
    if (why == 0)
      atomicOr(reinterpret_cast<unsigned long long*>(&a.present[gs]), 1ull << row);
    else if (why < 5)
      atomicAdd(&ctl[1 + why], 1u);
  }
  A ^= K;
  const uint32_t nx = from_next_lane(A.x), ny = from_next_lane(A.y);  // chunk m + 1 of the same packet
  const uint32_t o = 16u * m;
  if (lane == 63u || c >= total || why != 0 || o >= a.S) return;
  rx_put<1>(a.shards + row * a.rstride + gs * a.gstride, o, L, A, nx, ny);
}

}  // namespace kern
}  // namespace ugo
