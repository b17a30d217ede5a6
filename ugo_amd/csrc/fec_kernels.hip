// fec_kernels.hip -- gfx950 (CDNA4) kernels for batched GF(2^8) Reed-Solomon
// encode / erasure recovery: the arithmetic below reedsolomon.Encoder.Encode
// (ugo/fec.go:238) and .Reconstruct (ugo/fec.go:202).
//
// Work decomposition (DESIGN_HISTORY.md §3): a batch is shards[g][row][pitch].  One
// work item = one 16-byte column chunk of one group: the lane loads that chunk
// of each input row (global_load_dwordx4; consecutive lanes take consecutive
// chunks, so a wave's load of one row is 1 KiB contiguous), computes every
// output row's chunk in registers and stores it.  Each input byte is read from
// HBM exactly once and each output byte written once: the kernels are
// HBM-bound byte-field codecs, no MFMA.  The headline encode (k_encode_g)
// stages most of its row loads through LDS by LDS-DMA (global_load_lds_dwordx4
// nt, 1 KiB per row per wave); loads and stores are nontemporal, the policy
// that wins on a batch that is not in the Infinity Cache (DESIGN_HISTORY.md §3.4).
//
// GF(2^8) multiply-accumulate on 4 packed bytes per dword uses Horner's rule
// over the coefficient bits (bit 7 first):
//     y = (((T7 * 2) ^ T6) * 2 ^ ...) ^ T0,   Tb = XOR_{k : bit b of c_k} x_k
// so every output needs 7 "xtime" doublings regardless of the number of
// inputs, and the inputs enter only through XORs.  xtime on 4 bytes:
//     mask = v_perm_b32(y << 8, y, 0x090b080a)   (0xff in bytes whose bit 7 is
//            set: the sign-replicate selectors 8..11 read bytes 1,3 of y and of
//            y << 8)
//     xt   = ((y & 0x7f7f7f7f) << 1) ^ (mask & 0x1d1d1d1d)
//
//  * k_encode_c<D,P> / k_encode_g<D,P>: coefficients are compile-time
//    (gf::Code<D,P>), so the XOR network is fixed at compile time -- the (10,3)
//    headline (k_encode_g in production) and the (32,8) jumbo geometry
//    (k_encode_frs in production: the bit-plane sums Tb in Four-Russians form,
//    one precomputed XOR combination per block of inputs instead of one term
//    per input, dword by dword, for the VALU-bound wide code; gf_device.hpp
//    cparity_fr_seq).
//  * k_apply_p<DMAX,MODE>: runtime coefficients through split v_perm_b32
//    tables (the headline reconstruct), k_apply_q its streaming form for wide
//    codes, k_apply_qa the wave-aligned streaming form (the jumbo reconstruct:
//    rows just under a multiple of 64 chunks, one group per wave).
//  * k_apply<DMAX,MODE>: coefficients come from a *descriptor* (input rows,
//    output rows, e x d coefficient matrix).  MODE 0: one descriptor for all
//    groups (generic encode); MODE 1: descriptor table indexed by the group's
//    presence mask (d+p <= 16, built on the host at create time); MODE 2: one
//    descriptor per group written by k_prepare (larger codes).  A coefficient
//    bit becomes a lane mask with v_bfe_i32 and enters through v_bitop3
//    (y ^ (x & m)); the mask is reused for all 4 dwords of the chunk.
//  * k_apply_bytes<MODE>: any pitch / alignment / d, 4 columns per lane with
//    byte loads -- the correctness path for layouts the fast path rejects.
//  * Every reconstruct kernel writes output i (the i-th erased row) either in
//    place or, when Batch::out is set (ugo_fec_reconstruct_into), to slot i of
//    a separate output batch: then no row stream of the input mixes reads with
//    writes, 10% faster (DESIGN_HISTORY.md §3.4).
//  * k_prepare: per-group decode descriptor on device (first d present rows
//    -> d x d sub-matrix -> Gauss-Jordan in LDS -> reconstruct coefficients).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <utility>

#include "fec_kernels.hpp"
#include "gf256.hpp"
#include "gf_device.hpp"
#include "launch.hpp"

namespace ugo {
namespace kern {

// Location of work item `item` (group-local index gl, 16-byte chunk c).
struct Loc {
  uint8_t* gp;   // row 0, chunk c of the group
  uint32_t nb;   // valid bytes in the chunk (1..16)
};

__device__ __forceinline__ Loc locate(const Batch& a, uint32_t item) {
  const uint32_t gl = item / a.chunks;
  const uint32_t c = item - gl * a.chunks;
  return Loc{a.base + (a.g0 + gl) * a.gstride + static_cast<uint64_t>(c) * 16u, a.S - c * 16u};
}

// Destination of reconstruct output i (erased row r) for the chunk at byte
// offset `off` of group g: row r of the group itself (in place), or slot i of
// the caller's output batch (a.out: klauspost's Reconstruct hands erased, nil
// shards fresh buffers, ugo/fec.go:198-202).  a.out is a kernel argument, so
// the choice is a scalar branch.
__device__ __forceinline__ uint8_t* out_row(const Batch& a, uint8_t* gp, uint64_t g, uint32_t off, uint32_t r,
                                            uint32_t i) {
  return a.out ? a.out + g * a.ogstride + static_cast<uint64_t>(i) * a.orstride + off
               : gp + static_cast<uint64_t>(r) * a.rstride;
}

// List forms: entry g's output i at out + oent + i*orstride, where oent is
// the entry's offset -- row-compact (a.rowoff) or entry-strided.
__device__ __forceinline__ uint8_t* out_row_at(const Batch& a, uint8_t* gp, uint64_t oent, uint32_t off, uint32_t r,
                                              uint32_t i) {
  return a.out ? a.out + oent + static_cast<uint64_t>(i) * a.orstride + off : gp + static_cast<uint64_t>(r) * a.rstride;
}

template <int D, int NT>
__device__ __forceinline__ void load_rows(V4* x, const uint8_t* gp, uint64_t rstride) {
#pragma unroll
  for (int k = 0; k < D; ++k) x[k] = load16<NT>(gp + static_cast<uint64_t>(k) * rstride);
}

// One 16-byte column chunk per thread over a full grid (items / 256 blocks).
// Measured on MI355X (tools/kvariants.hip, DESIGN_HISTORY.md §4): a full grid at
// 8 waves/SIMD (62 VGPRs) beats persistent grids and software-pipelined
// (ping-pong) forms, whose second register set halves occupancy.
template <int D, int P, int NT, int SWZ = 0>
__global__ __launch_bounds__(256) void k_encode_c(Batch a) {
  const uint32_t item = block_id<SWZ>() * 256u + threadIdx.x;
  if (item >= a.items) return;
  const Loc l = locate(a, item);
  V4 x[D];
  load_rows<D, NT>(x, l.gp, a.rstride);
  cparity_store<D, P, NT>(l.gp, a.rstride, l.nb, x, std::make_integer_sequence<int, P>{});
}

// k_encode_c with the first GR row loads staged through LDS by LDS-DMA (nt)
// and the rest loaded to registers (nt): each wave owns GR x 1 KiB of LDS.
// LR >= GR sizes the stage, and with it the blocks per CU: the (10,3) encode
// stages 8 rows in a 13-row stage (52 KiB per block), which caps it at 3
// blocks = 3 waves per SIMD.  Fewer requests in flight run the 10-read +
// 3-write stream mix faster on a cold batch: 188.6 us at 3 blocks/CU against
// 194.9 at 4, 194.7 at 5 (the 8-row stage's natural occupancy) and 193.1 at
// 2; in the bench's encode + reconstruct step 366.0 against 372.0 us
// (profiles/r2/kvar_cold_occupancy_exact.jsonl).
template <int D, int P, int NTS = 0, int GR = D, int BS = 256, int LR = GR>
__global__ __launch_bounds__(BS) void k_encode_g(Batch a) {
  static_assert(LR >= GR, "the stage holds at least the staged rows");
  __shared__ u32x4 stage[BS / 64][LR][64];
  const uint32_t item = blockIdx.x * BS + threadIdx.x;
  if (item >= a.items) return;
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const Loc l = locate(a, item);
#pragma unroll
  for (int k = 0; k < GR; ++k) lds_dma16(l.gp + static_cast<uint64_t>(k) * a.rstride, &stage[w][k][0]);
  V4 x[D];
#pragma unroll
  for (int k = GR; k < D; ++k) x[k] = load16<1>(l.gp + static_cast<uint64_t>(k) * a.rstride);
  lds_dma_wait();
#pragma unroll
  for (int k = 0; k < GR; ++k) x[k] = lds16(&stage[w][k][lane]);
  cparity_store<D, P, NTS>(l.gp, a.rstride, l.nb, x, std::make_integer_sequence<int, P>{});
}

// k_encode_fr with the dwords forced in sequence (cparity_fr_seq): staged rows
// read from LDS per dword, so the live set is one dword's tables.
// XCD (grid a multiple of 8): block b works on tile (b % 8) * (grid / 8) + b / 8,
// each XCD on one contiguous eighth of the batch (k_apply_qb OPT & 32).
template <int D, int P, int NTS = 0, int GR = D, int BS = 256, int LR = GR, int WPE = 1, int BK = kFrBlock,
          bool XCD = false>
__global__ __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(WPE))) void k_encode_frs(Batch a) {
  static_assert(LR >= GR, "the stage holds at least the staged rows");
  __shared__ u32x4 stage[BS / 64][LR][64];
  uint32_t bid = blockIdx.x;
  if constexpr (XCD) bid = (blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  const uint32_t item = bid * BS + threadIdx.x;
  if (item >= a.items) return;
  const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const Loc l = locate(a, item);
#pragma unroll
  for (int k = 0; k < GR; ++k) lds_dma16(l.gp + static_cast<uint64_t>(k) * a.rstride, &stage[w][k][0]);
  V4 x[D];
#pragma unroll
  for (int k = GR; k < D; ++k) x[k] = load16<1>(l.gp + static_cast<uint64_t>(k) * a.rstride);
  lds_dma_wait();
  V4 y[P];
  cparity_fr_seq<D, P, GR, BK>(y, x, reinterpret_cast<const uint32_t*>(&stage[w][0][lane]));
#pragma unroll
  for (int i = 0; i < P; ++i) store16<NTS>(l.gp + static_cast<uint64_t>(D + i) * a.rstride, y[i], l.nb);
}

// ----------------------------------------------- descriptor-driven kernels
// Descriptor (DESIGN_HISTORY.md §3.3), byte offsets:
//   [0] e_total  [1] e_data  [2] status  [3] reserved
//   [4, 4+dpad)            input rows (survivors / data rows)
//   [4+dpad, 4+dpad+epad)  output rows: erased data rows, then erased parity
//   [4+dpad+epad + i*dpad] coefficient row i (d bytes, zero padded)
template <int MODE>
__device__ __forceinline__ const uint8_t* desc_for(const Batch& a, uint64_t g) {
  if constexpr (MODE == 0) {
    return a.desc;
  } else if constexpr (MODE == 1) {
    const uint64_t m = a.present[g] & a.nmask;
    return a.desc + m * a.desc_stride;
  } else {
    return a.desc + (g - a.g_desc0) * a.desc_stride;
  }
}


// List form: the launch's work items over the list entries [g0, *count).
__device__ __forceinline__ uint32_t list_items(const Batch& a) {
  const uint64_t cnt = *a.count;
  if (cnt <= a.g0) return 0u;
  return static_cast<uint32_t>(min(static_cast<uint64_t>(a.items), (cnt - a.g0) * a.chunks));
}

// One 16-byte chunk per thread over a full grid; the descriptor (presence
// mask -> table entry, or the group's workspace entry) is read per thread from
// L2.  Staging descriptors per tile in LDS and software-pipelining the next
// item measured slower (fewer waves per SIMD), see DESIGN_HISTORY.md §4.
template <int DMAX, int MODE, int NT, bool LIST = false>
__global__ __launch_bounds__(256) void k_apply(Batch a) {
  const uint32_t item = blockIdx.x * 256u + threadIdx.x;
  uint32_t items = a.items;
  if constexpr (LIST) items = list_items(a);
  if (item >= items) return;
  const uint32_t gl = item / a.chunks;
  const uint32_t c = item - gl * a.chunks;
  const uint64_t g = a.g0 + gl;  // output / status index (list entry in the list form)
  const uint64_t grow = LIST ? a.list[g] : g;  // the group whose rows are read
  const uint8_t* desc = desc_for<MODE>(a, grow);
  const uint32_t hdr = ld32(desc);
  const uint32_t st = (hdr >> 16) & 0xffu;
  if (MODE != 0 && a.status != nullptr && c == 0) a.status[g] = static_cast<int8_t>(st);
  const uint32_t e = a.data_only ? ((hdr >> 8) & 0xffu) : (hdr & 0xffu);
  if (st != 0 || e == 0) return;
  uint8_t* gp = a.base + grow * a.gstride + static_cast<uint64_t>(c) * 16u;
  const uint32_t rbase = LIST && a.rowoff ? a.rowoff[g] : 0u;  // row-compact: the entry's first output row
  const uint64_t oent = !LIST ? g * a.ogstride : a.rowoff ? uint64_t(rbase) * a.orstride : g * a.ogstride;
  constexpr int NW = (DMAX + 3) / 4;
  uint32_t rows[NW];
#pragma unroll
  for (int w = 0; w < NW; ++w) rows[w] = ld32(desc + 4 + 4 * w);
  V4 x[DMAX];
#pragma unroll
  for (int k = 0; k < DMAX; ++k) {
    if (k < static_cast<int>(a.d)) {
      const uint32_t r = (rows[k >> 2] >> (8 * (k & 3))) & 0xffu;
      x[k] = load16<NT>(gp + static_cast<uint64_t>(r) * a.rstride);
    } else {
      x[k] = V4{{0u, 0u, 0u, 0u}};
    }
  }
  const uint32_t nb = a.S - c * 16u;
  const uint8_t* orow = desc + 4 + a.dpad;
  const uint8_t* coef = orow + a.epad;
  for (uint32_t i = 0; i < e; ++i) {
    uint32_t cw[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) cw[w] = ld32(coef + i * a.dpad + 4 * w);
    const V4 y = horner_var<DMAX>(x, cw);
    if (LIST && a.rowoff && rbase + i >= a.max_rows) break;  // rows past the caller's room
    store16<NT>(out_row_at(a, gp, oent, c * 16u, orow[i], i), y, nb);
    if (LIST && a.rowid && c == 0) a.rowid[rbase + i] = static_cast<uint32_t>(grow * a.n + orow[i]);
  }
}

// Wave-scalar form, for rows of >= 64 chunks (S > 1008 B): a 64-lane wave
// then spans at most two groups, A and B = A + 1.  Both groups' presence masks
// and descriptors are fetched with scalar loads (wave-uniform addresses), and
// each lane selects its group's words with v_cndmask.  This removes the
// per-lane mask -> descriptor -> data dependent vector-load chain of k_apply
// and the per-lane descriptor loads (DESIGN_HISTORY.md §4).
//
// CPT > 1: a thread owns CPT chunks `a.pass` items apart (a.pass % 64 == 0, so
// every range is still wave-aligned); all CPT sets of survivor loads are
// issued before the first chunk's arithmetic, so later chunks' data arrives
// while earlier ones compute.
template <int DMAX>
struct WItem {
  const uint8_t* dA;
  const uint8_t* dB;
  uint8_t* gp;
  uint64_t g;
  uint32_t c, nb, e, orows;
  bool inB, live;
  V4 x[DMAX];
};

template <int DMAX, int MODE, int NT>
__device__ __forceinline__ void witem_issue(WItem<DMAX>& it, const Batch& a, uint32_t wfirst, uint32_t item) {
  it.live = false;
  if (wfirst >= a.items) return;
  const uint32_t wlast = min(wfirst + 63u, a.items - 1u);
  const uint32_t gA = wfirst / a.chunks;
  const uint32_t gB = wlast / a.chunks;  // gA or gA + 1
  it.dA = desc_for<MODE>(a, a.g0 + gA);
  it.dB = desc_for<MODE>(a, a.g0 + gB);
  constexpr int NW = (DMAX + 3) / 4;
  const uint32_t hA = ld32(it.dA), hB = ld32(it.dB);
  uint32_t rA[NW], rB[NW];
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    rA[w] = ld32(it.dA + 4 + 4 * w);
    rB[w] = ld32(it.dB + 4 + 4 * w);
  }
  const uint32_t oA = ld32(it.dA + 4 + a.dpad), oB = ld32(it.dB + 4 + a.dpad);  // output rows (e <= 4)
  if (item >= a.items) return;
  const uint32_t gl = item / a.chunks;
  it.inB = gl != gA;
  const uint32_t c = item - gl * a.chunks;
  const uint64_t g = a.g0 + gl;
  const uint32_t hdr = it.inB ? hB : hA;
  const uint32_t st = (hdr >> 16) & 0xffu;
  if (MODE != 0 && a.status != nullptr && c == 0) a.status[g] = static_cast<int8_t>(st);
  it.e = a.data_only ? ((hdr >> 8) & 0xffu) : (hdr & 0xffu);
  if (st != 0 || it.e == 0) return;
  it.live = true;
  it.gp = a.base + g * a.gstride + static_cast<uint64_t>(c) * 16u;
  it.g = g;
  it.c = c;
  it.nb = a.S - c * 16u;
  it.orows = it.inB ? oB : oA;
#pragma unroll
  for (int k = 0; k < DMAX; ++k) {
    if (k < static_cast<int>(a.d)) {
      const uint32_t rw = it.inB ? rB[k >> 2] : rA[k >> 2];
      const uint32_t r = (rw >> (8 * (k & 3))) & 0xffu;
      it.x[k] = load16<NT>(it.gp + static_cast<uint64_t>(r) * a.rstride);
    } else {
      it.x[k] = V4{{0u, 0u, 0u, 0u}};
    }
  }
}

template <int DMAX, int NT>
__device__ __forceinline__ void witem_finish(const WItem<DMAX>& it, const Batch& a) {
  if (!it.live) return;
  constexpr int NW = (DMAX + 3) / 4;
  const uint32_t cbase = 4 + a.dpad + a.epad;
  for (uint32_t i = 0; i < it.e; ++i) {
    uint32_t cw[NW];
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const uint32_t ca = ld32(it.dA + cbase + i * a.dpad + 4 * w);
      const uint32_t cb = ld32(it.dB + cbase + i * a.dpad + 4 * w);
      cw[w] = it.inB ? cb : ca;
    }
    const V4 y = horner_var<DMAX>(it.x, cw);
    const uint32_t r = (it.orows >> (8 * i)) & 0xffu;
    store16<NT>(out_row(a, it.gp, it.g, it.c * 16u, r, i), y, it.nb);
  }
}

template <int DMAX, int MODE, int NT, int CPT = 1>
__global__ __launch_bounds__(256) void k_apply_w(Batch a) {
  const uint32_t wfirst = blockIdx.x * 256u + (__builtin_amdgcn_readfirstlane(threadIdx.x) & ~63u);
  const uint32_t item = blockIdx.x * 256u + threadIdx.x;
  WItem<DMAX> it[CPT];
#pragma unroll
  for (int j = 0; j < CPT; ++j) witem_issue<DMAX, MODE, NT>(it[j], a, wfirst + j * a.pass, item + j * a.pass);
#pragma unroll
  for (int j = 0; j < CPT; ++j) witem_finish<DMAX, NT>(it[j], a);
}

// Table form of the wave-scalar kernel.  The masked Horner of k_apply_w costs
// 8 * (d + 4) ops per output dword (+ mask extraction); here each product
// c * x is three v_perm_b32 lookups into 8-byte split tables of c
// (gf::perm_tables): T0[x & 7] ^ T1[(x >> 3) & 7] ^ T2[x >> 6].  The selector
// bytes of an input are extracted once and shared by all outputs (inputs
// outer, outputs inner, accumulators live), and a coefficient's five table
// dwords come from the scalar cache (8 KiB table), selected per lane between
// the wave's two groups.  Output rows beyond a group's e get coefficient 0
// (zero tables) and are not stored.

// TSEL: how a lane gets its group's tables when the wave spans groups A, B.
//   0: wave-uniform (dA == dB), scalar loads only
//   1: scalar loads of both, per-lane pick as arithmetic
//   2: per-lane vector loads of the picked group's table (L1-resident)
template <int TSEL>
__device__ __forceinline__ void p_tables(uint32_t* t, const Batch& a, const uint8_t* dA, const uint8_t* dB,
                                         uint32_t off, int k, uint32_t mB) {
  const uint32_t cA = (ld32(dA + off) >> (8 * (k & 3))) & 0xffu;
  const uint32_t* tA = a.mult + 8u * cA;
  if constexpr (TSEL == 0) {
#pragma unroll
    for (int q = 0; q < 5; ++q) t[q] = tA[q];
  } else {
    const uint32_t cB = (ld32(dB + off) >> (8 * (k & 3))) & 0xffu;
    const uint32_t* tB = a.mult + 8u * cB;
    if constexpr (TSEL == 1) {
#pragma unroll
      for (int q = 0; q < 5; ++q) {  // vA ^ ((vA ^ vB) & mB): the XOR of the two scalar
        const uint32_t va = tA[q];   // words is SALU work, the pick two VALU ops with one
        const uint32_t vb = tB[q];   // SGPR each (mB is opaque, so this is not rewritten
        t[q] = va ^ ((va ^ vb) & mB);  // into a select / per-lane vector load)
      }
    } else {
      const uint32_t* tp = mB ? tB : tA;
#pragma unroll
      for (int q = 0; q < 5; ++q) t[q] = tp[q];
    }
  }
}

// Word loads through the constant address space: they stay scalar loads even
// after stores to global memory in the same kernel (a plain load there loses
// its no-clobber proof and becomes a per-lane vector load).  Descriptors and
// tables are never written by a kernel that reads them.
typedef const __attribute__((address_space(4))) uint32_t* ctab_t;

template <bool C>
__device__ __forceinline__ uint32_t ldw(const uint8_t* p) {
  if constexpr (C)
    return *(ctab_t)(p);
  else
    return ld32(p);
}

// p_tables for a wave-uniform descriptor, constant-space loads when C
template <bool C>
__device__ __forceinline__ void p_tables_u(uint32_t* t, const Batch& a, const uint8_t* dS, uint32_t off, int k) {
  const uint32_t c = (ldw<C>(dS + off) >> (8 * (k & 3))) & 0xffu;
  if constexpr (C) {
    const ctab_t tA = (ctab_t)(a.mult) + 8u * c;
#pragma unroll
    for (int q = 0; q < 5; ++q) t[q] = tA[q];
  } else {
    const uint32_t* tA = a.mult + 8u * c;
#pragma unroll
    for (int q = 0; q < 5; ++q) t[q] = tA[q];
  }
}

__device__ __forceinline__ void p_sel(const V4& x, uint32_t* s0, uint32_t* s1, uint32_t* s2) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    s0[j] = x.v[j] & 0x07070707u;
    s1[j] = (x.v[j] >> 3) & 0x07070707u;
    s2[j] = (x.v[j] >> 6) & 0x03030303u;
  }
}

// TSEL: how a lane gets its group's tables when the wave spans groups A, B.
//   0: wave-uniform (dA == dB), scalar loads only
//   1: scalar loads of both, per-lane pick as arithmetic
//   2: per-lane vector loads of the picked group's table (L1-resident)
// Inputs are taken in pairs so that the six table lookups of two products fold
// into an accumulator with three xor3 (DMAX is even; a missing odd input is a
// zero chunk, whose lookups are zero whatever the coefficient).
template <int DMAX, int TSEL, int EMAX, bool PAIR>
__device__ __forceinline__ void p_accum(V4* acc, const V4* x, const Batch& a, const uint8_t* dA,
                                        const uint8_t* dB, uint32_t mB, uint32_t emax) {
  static_assert(DMAX % 2 == 0 || !PAIR, "inputs are taken in pairs");
#pragma unroll
  for (int i = 0; i < EMAX; ++i) acc[i] = V4{{0u, 0u, 0u, 0u}};
  const uint32_t cbase = 4 + a.dpad + a.epad;
  constexpr int KS = PAIR ? 2 : 1;
#pragma unroll
  for (int k = 0; k < DMAX; k += KS) {
    if (k >= static_cast<int>(a.d)) continue;
    uint32_t s0[4], s1[4], s2[4], r0[4], r1[4], r2[4];
    p_sel(x[k], s0, s1, s2);
    if constexpr (PAIR) p_sel(x[k + 1], r0, r1, r2);
#pragma unroll
    for (int i = 0; i < EMAX; ++i) {
      if (i >= static_cast<int>(emax)) continue;
      const uint32_t off = cbase + i * a.dpad + (k & ~3);
      uint32_t t[5], u[5];
      p_tables<TSEL>(t, a, dA, dB, off, k, mB);
      if constexpr (PAIR) {
        p_tables<TSEL>(u, a, dA, dB, off, k + 1, mB);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          uint32_t y = xor3(acc[i].v[j], perm(t[1], t[0], s0[j]), perm(t[3], t[2], s1[j]));
          y = xor3(y, perm(0u, t[4], s2[j]), perm(u[1], u[0], r0[j]));
          acc[i].v[j] = xor3(y, perm(u[3], u[2], r1[j]), perm(0u, u[4], r2[j]));
        }
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i].v[j] = xor3(acc[i].v[j], perm(t[1], t[0], s0[j]), perm(t[3], t[2], s1[j])) ^
                        perm(0u, t[4], s2[j]);
      }
    }
  }
}

template <int DMAX, int MODE, int NT, int TSEL = 1, int WPE = 1, int EMAX = 4, bool PAIR = true, int SWZ = 0,
          int GLR = 0, bool LIST = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_apply_p(Batch a) {
  // GLR > 0 (A/B only): survivors 0..GLR-1 by LDS-DMA nt.  It ties register
  // loads on a cold batch (201.0 vs 201.0 us) and in a warm loop (187.3 vs
  // 188.0 us): DESIGN_HISTORY.md §3.4.
  static_assert(GLR == 0 || (DMAX == 10 && (GLR == 8 || GLR == 10)), "LDS-DMA survivor staging: d = 10");
  __shared__ u32x4 stage[GLR ? 4 : 1][GLR ? GLR : 1][64];
  const uint32_t bid = block_id<SWZ>();
  const uint32_t wfirst = bid * 256u + (__builtin_amdgcn_readfirstlane(threadIdx.x) & ~63u);
  const uint32_t item = bid * 256u + threadIdx.x;
  uint32_t items = a.items;
  if constexpr (LIST) items = list_items(a);  // list form: entries past *count idle
  if (wfirst >= items) return;
  const uint32_t wlast = min(wfirst + 63u, items - 1u);
  const uint32_t gA = wfirst / a.chunks;
  const uint32_t gB = wlast / a.chunks;
  uint64_t rA = a.g0 + gA, rB = a.g0 + gB;  // the wave's (at most) two groups whose rows it reads
  if constexpr (LIST) {
    rA = a.list[rA];
    rB = a.list[rB];
  }
  const uint8_t* dA = desc_for<MODE>(a, rA);
  const uint8_t* dB = desc_for<MODE>(a, rB);
  constexpr int NW = (DMAX + 3) / 4;
  const uint32_t hA = ld32(dA), hB = ld32(dB);
  uint32_t wA[NW], wB[NW];  // survivor row words
#pragma unroll
  for (int w = 0; w < NW; ++w) {
    wA[w] = ld32(dA + 4 + 4 * w);
    wB[w] = ld32(dB + 4 + 4 * w);
  }
  const uint32_t oA = ld32(dA + 4 + a.dpad), oB = ld32(dB + 4 + a.dpad);
  // wave-uniform output count: the larger of the two groups' (a failed group
  // contributes nothing: its lanes leave below)
  const uint32_t eA = ((hA >> 16) & 0xffu) ? 0u : (a.data_only ? ((hA >> 8) & 0xffu) : (hA & 0xffu));
  const uint32_t eB = ((hB >> 16) & 0xffu) ? 0u : (a.data_only ? ((hB >> 8) & 0xffu) : (hB & 0xffu));
  const uint32_t emax = max(eA, eB);
  if (item >= items) return;
  const uint32_t gl = item / a.chunks;
  const bool inB = gl != gA;
  const uint32_t c = item - gl * a.chunks;
  const uint64_t g = a.g0 + gl;  // output / status index (list entry in the list form)
  const uint64_t grow = LIST ? (inB ? rB : rA) : g;
  const uint32_t hdr = inB ? hB : hA;
  const uint32_t st = (hdr >> 16) & 0xffu;
  // (the status store comes last: a vector store ahead of the table reads
  // would stop them being scalar loads)
  const bool wst = MODE != 0 && a.status != nullptr && c == 0;
  const uint32_t e = inB ? eB : eA;
  if (e == 0) {
    if (wst) a.status[g] = static_cast<int8_t>(st);
    return;
  }
  uint32_t mB;  // all-ones in group-B lanes; opaque to the optimizer (see p_tables)
  asm("v_mov_b32 %0, %1" : "=v"(mB) : "v"(inB ? ~0u : 0u));
  uint8_t* gp = a.base + grow * a.gstride + static_cast<uint64_t>(c) * 16u;
  const uint32_t rbase = LIST && a.rowoff ? a.rowoff[g] : 0u;  // row-compact: the entry's first output row
  const uint64_t oent = !LIST ? g * a.ogstride : a.rowoff ? uint64_t(rbase) * a.orstride : g * a.ogstride;
  const uint32_t nb = a.S - c * 16u;
  V4 x[DMAX];
  if constexpr (GLR > 0) {  // survivors 0..GLR-1 by LDS-DMA nt, the rest to registers (host: d == 10)
    const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
    const uint32_t sbase = lds_addr(&stage[w][0][0]);
    uint32_t tok = 0;
#pragma unroll
    for (int k = 0; k < DMAX; ++k) {
      const uint32_t rw = inB ? wB[k >> 2] : wA[k >> 2];
      const uint32_t r = (rw >> (8 * (k & 3))) & 0xffu;
      if (k < GLR)
        lds_dma16_nt_asm(gp + static_cast<uint64_t>(r) * a.rstride, sbase + 1024u * k, tok);
      else
        x[k] = load16<NT>(gp + static_cast<uint64_t>(r) * a.rstride);
    }
    lds_collect<GLR>(x, &stage[w][0][lane], tok);
  } else {
#pragma unroll
    for (int k = 0; k < DMAX; ++k) {
      if (k < static_cast<int>(a.d)) {
        const uint32_t rw = inB ? wB[k >> 2] : wA[k >> 2];
        const uint32_t r = (rw >> (8 * (k & 3))) & 0xffu;
        x[k] = load16<NT>(gp + static_cast<uint64_t>(r) * a.rstride);
      } else {
        x[k] = V4{{0u, 0u, 0u, 0u}};
      }
    }
  }
  V4 acc[EMAX];
  if (dA == dB)  // one descriptor for the whole wave: no per-lane table pick
    p_accum<DMAX, 0, EMAX, PAIR>(acc, x, a, dA, dA, 0u, emax);
  else
    p_accum<DMAX, TSEL, EMAX, PAIR>(acc, x, a, dA, dB, mB, emax);
  const uint32_t orows = inB ? oB : oA;
#pragma unroll
  for (int i = 0; i < EMAX; ++i) {
    if (i >= static_cast<int>(e)) continue;
    const uint32_t r = (orows >> (8 * i)) & 0xffu;
    if (LIST && a.rowoff && rbase + i >= a.max_rows) continue;  // rows past the caller's room
    store16<NT>(out_row_at(a, gp, oent, c * 16u, r, i), acc[i], nb);
    if (LIST && a.rowid && c == 0) a.rowid[rbase + i] = static_cast<uint32_t>(grow * a.n + r);
  }
  if (wst) a.status[g] = 0;
}

// k_apply_p for DENSE rows (group stride == S, no padding: row r of group g at
// base + r*rstride + g*S, rows 16-B aligned, S >= 1009).  Lanes take the rows'
// aligned 16-B chunks, not per-group ones, so every load and store is aligned.
// Before this kernel dense rows ran the byte kernel.  On the (10,3) bench step
// it takes 186-189 us against 172-178 for k_apply_p on the 16-B pitch (the two
// partial stores of each straddling chunk ~9 us, the idle 64th lane ~3 us;
// k_apply_p on 2-B aligned groups: 186-189 too; profiles/r3/dense/), so the
// bench keeps padded rows.  A wave covers 63 chunks (1008 B < S: at most one group
// boundary EB, groups A and B as in k_apply_p); a chunk's group is the group
// of its first byte.  When EB is not 16-B aligned its chunk holds the end of
// A and the start of B: that lane stores A's bytes [0, EB % 16), and lane 63
// -- a B lane on the same chunk, B's rows and B's tables, in the same
// instructions as every other lane -- stores B's bytes [EB % 16, 16).  The
// group's status goes with the lane that holds its first byte.
__device__ __forceinline__ void store16_from(uint8_t* p, const V4& y, uint32_t lo) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t b0 = 4u * j, w = y.v[j];
    if (lo <= b0) {
      *reinterpret_cast<uint32_t*>(p + b0) = w;
    } else if (lo < b0 + 4) {
      if (lo <= b0 + 1) p[b0 + 1] = static_cast<uint8_t>(w >> 8);
      if (lo <= b0 + 2) p[b0 + 2] = static_cast<uint8_t>(w >> 16);
      p[b0 + 3] = static_cast<uint8_t>(w >> 24);
    }
  }
}

template <int DMAX, int MODE, int NT, int EMAX = 4>
__global__ __launch_bounds__(256) void k_apply_pd(Batch a) {
  // a.base: row 0 of group a.g0 (16-B aligned); a.items: the slice's aligned
  // chunks per row, ceil(groups * S / 16); a.n: groups in the slice
  const uint32_t w = blockIdx.x * 4u + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t c0 = w * 63u;  // the wave's first chunk
  if (c0 >= a.items) return;
  const uint32_t S = a.S;
  const uint64_t fw = static_cast<uint64_t>(c0) * 16u;
  const uint32_t gA = static_cast<uint32_t>(fw / S);
  const uint64_t eb = static_cast<uint64_t>(gA + 1u) * S;  // end of group A
  const uint32_t cend = min(c0 + 63u, a.items);
  const bool has_b = gA + 1u < a.n && eb < static_cast<uint64_t>(cend) * 16u;
  const uint32_t gB = has_b ? gA + 1u : gA;
  const uint8_t* dA = desc_for<MODE>(a, a.g0 + gA);
  const uint8_t* dB = desc_for<MODE>(a, a.g0 + gB);
  constexpr int NW = (DMAX + 3) / 4;
  const uint32_t hA = ld32(dA), hB = ld32(dB);
  uint32_t rA[NW], rB[NW];
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    rA[q] = ld32(dA + 4 + 4 * q);
    rB[q] = ld32(dB + 4 + 4 * q);
  }
  const uint32_t oA = ld32(dA + 4 + a.dpad), oB = ld32(dB + 4 + a.dpad);
  const uint32_t eA = ((hA >> 16) & 0xffu) ? 0u : (a.data_only ? ((hA >> 8) & 0xffu) : (hA & 0xffu));
  const uint32_t eB = ((hB >> 16) & 0xffu) ? 0u : (a.data_only ? ((hB >> 8) & 0xffu) : (hB & 0xffu));
  const uint32_t emax = max(eA, eB);
  // this lane's chunk, group and byte range [lo, hi) of the chunk it stores
  uint64_t f;
  bool inB;
  uint32_t lo = 0, hi;
  if (lane < 63u) {
    const uint32_t ci = c0 + lane;
    if (ci >= a.items) return;
    f = static_cast<uint64_t>(ci) * 16u;
    inB = has_b && f >= eb;
    const uint64_t gend = inB ? eb + S : eb;  // end of this lane's group
    hi = static_cast<uint32_t>(min(gend - f, static_cast<uint64_t>(16)));
  } else {  // lane 63: B's bytes of a straddling chunk, if any
    if (!has_b || (eb & 15u) == 0) return;
    f = eb & ~static_cast<uint64_t>(15);
    inB = true;
    lo = static_cast<uint32_t>(eb & 15u);
    hi = 16u;
  }
  const uint64_t gstart = inB ? eb : eb - S;
  const uint64_t g = a.g0 + (inB ? gB : gA);
  const uint32_t hdr = inB ? hB : hA;
  const uint32_t st = (hdr >> 16) & 0xffu;
  const bool wst = a.status != nullptr && f <= gstart && gstart < f + 16u;  // holds the group's first byte
  const uint32_t e = inB ? eB : eA;
  if (e == 0) {
    if (wst) a.status[g] = static_cast<int8_t>(st);
    return;
  }
  uint32_t mB;
  asm("v_mov_b32 %0, %1" : "=v"(mB) : "v"(inB ? ~0u : 0u));
  uint8_t* gp = a.base + f;
  V4 x[DMAX];
#pragma unroll
  for (int k = 0; k < DMAX; ++k) {
    if (k < static_cast<int>(a.d)) {
      const uint32_t rw = inB ? rB[k >> 2] : rA[k >> 2];
      const uint32_t r = (rw >> (8 * (k & 3))) & 0xffu;
      x[k] = load16<NT>(gp + static_cast<uint64_t>(r) * a.rstride);
    } else {
      x[k] = V4{{0u, 0u, 0u, 0u}};
    }
  }
  V4 acc[EMAX];
  if (dA == dB)
    p_accum<DMAX, 0, EMAX, true>(acc, x, a, dA, dA, 0u, emax);
  else
    p_accum<DMAX, 1, EMAX, true>(acc, x, a, dA, dB, mB, emax);
  const uint32_t orows = inB ? oB : oA;
  const int64_t off = static_cast<int64_t>(f) - static_cast<int64_t>(gstart);  // chunk start within the group
#pragma unroll
  for (int i = 0; i < EMAX; ++i) {
    if (i >= static_cast<int>(e)) continue;
    const uint32_t r = (orows >> (8 * i)) & 0xffu;
    uint8_t* p = a.out ? a.out + static_cast<int64_t>(g * a.ogstride + static_cast<uint64_t>(i) * a.orstride) + off
                       : gp + static_cast<uint64_t>(r) * a.rstride;
    if (lo)
      store16_from(p, acc[i], lo);
    else  // (a partial chunk's stores take any byte address: an output batch of any layout)
      store16<NT>(p, acc[i], hi);
  }
  if (wst) a.status[g] = 0;
}

// ---------------------------------------------------------------- per-call service
// k_service: ONE block of 8 waves stays resident and serves the per-group
// calls of the drop-in path (one Encode from calcECC, one Reconstruct per lossy
// group from input: ugo/fec.go:202,238) from a mailbox in pinned host memory
// (SvcBox, fec_kernels.hpp).  Thread 0 polls the request word with relaxed
// system-scope loads and s_sleep, then ONE system-scope acquire; the block
// reads the batch's rows over PCIe, applies the descriptor (the encode
// descriptor, or the MODE-1 table entry of each group's presence mask) with
// the same split-table products as k_apply_p, one group per wave at a time,
// and writes the outputs back through the mapping.  Every wave drains its
// stores, the block meets, and thread 0 releases at system scope and stores
// done = seq.  Exit: idle_ticks without a request, or a stop request; `alive`
// is cleared last.  All stores are vector stores.
// Global-address-space 16-B access for the service: a flat access would also
// count in lgkmcnt, so every scalar descriptor wait would wait for the PCIe
// round trips of the loads before it.
typedef __attribute__((address_space(1))) u32x4 g_u32x4;
typedef __attribute__((address_space(1))) uint32_t g_u32;
typedef __attribute__((address_space(1))) uint8_t g_u8;

__device__ __forceinline__ V4 gload16(const uint8_t* p) {
  const u32x4 v = *(const g_u32x4*)(p);
  return V4{{v.x, v.y, v.z, v.w}};
}

__device__ __forceinline__ void gstore16(uint8_t* p, const V4& y, uint32_t nb) {
  if (nb >= 16) {
    *(g_u32x4*)(p) = u32x4{y.v[0], y.v[1], y.v[2], y.v[3]};
    return;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t lo = 4u * j;
    if (nb >= lo + 4) {
      *(g_u32*)(p + lo) = y.v[j];
    } else if (nb > lo) {
      const uint32_t w = y.v[j], rem = nb - lo;
      *(g_u8*)(p + lo) = static_cast<uint8_t>(w);
      if (rem >= 2) *(g_u8*)(p + lo + 1) = static_cast<uint8_t>(w >> 8);
      if (rem >= 3) *(g_u8*)(p + lo + 2) = static_cast<uint8_t>(w >> 16);
    }
  }
}

// The service keeps its tables in LDS: the split-table words of all 256
// coefficients (copied once at start) and, per slot (a group of the request,
// or the encode slot copied at start), the descriptor itself.  A request's
// descriptors are ONE round of parallel loads; every table lookup after that
// is an LDS read, where reading them through the scalar cache would be a
// chain of dependent loads per product.
constexpr uint32_t kSvcDescWords = 32;  // descriptor bytes <= 128 (host: svc_eligible)
template <int DMAX>
struct SvcLds {
  uint32_t mult[256][5];                         // split tables of every coefficient
  uint32_t desc[kSvcMaxGroups + 1][kSvcDescWords];
  uint32_t t[kSvcMaxGroups + 1][4][DMAX][5];     // per slot: tables of every (output, input) product
  u32x4 rows[DMAX][128];                         // one-group requests: the survivors' chunks
};

template <int DMAX>
__device__ __forceinline__ void svc_copy_desc(SvcLds<DMAX>& L, uint32_t slot, const uint8_t* desc, uint32_t words,
                                              uint32_t tid, uint32_t nthreads) {
  for (uint32_t w = tid; w < words; w += nthreads) L.desc[slot][w] = *(const g_u32*)(desc + 4u * w);
}

// the slot's product tables from its descriptor copy and the LDS mult table
template <int DMAX>
__device__ __forceinline__ void svc_expand(SvcLds<DMAX>& L, uint32_t slot, const Batch& a, uint32_t tid,
                                           uint32_t nthreads) {
  for (uint32_t it = tid; it < 4u * DMAX * 5u; it += nthreads) {
    const uint32_t q = it % 5u, k = (it / 5u) % DMAX, i = it / (5u * DMAX);
    const uint32_t off = 4u + a.dpad + a.epad + i * a.dpad + k;
    const uint32_t c = (L.desc[slot][off / 4u] >> (8u * (off & 3u))) & 0xffu;
    L.t[slot][i][k][q] = L.mult[c][q];
  }
}

#ifndef UGO_SVC_SLEEP  // the poll's s_sleep between reads of the request line (A/B builds only)
#define UGO_SVC_SLEEP 1
#endif
constexpr uint32_t kSvcThreads = 512;  // 8 waves: 2 per SIMD, so DMAX 16 fits its registers

template <int DMAX>
__global__ __launch_bounds__(kSvcThreads) void k_service(SvcArgs sa) {
  static_assert(DMAX % 2 == 0, "inputs are taken in pairs");
  __shared__ u32x4 line[4];                     // the request line
  __shared__ uint64_t msk[kSvcMaxGroups];       // presence masks of a reconstruct
  __shared__ SvcLds<DMAX> L;
  constexpr uint32_t ENC = kSvcMaxGroups;  // the encode slot
  SvcBox* box = sa.box;
  const Batch& a = sa.a;
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t dwords = a.desc_stride / 4u;
  for (uint32_t w = threadIdx.x; w < 256u * 5u; w += kSvcThreads) L.mult[w / 5u][w % 5u] = a.mult[8u * (w / 5u) + w % 5u];
  svc_copy_desc(L, ENC, sa.encdesc, dwords, threadIdx.x, kSvcThreads);
  __syncthreads();
  svc_expand(L, ENC, a, threadIdx.x, kSvcThreads);
  uint32_t last = sa.start_seq;
  uint64_t t0 = wall_clock64();
#ifdef UGO_SVC_TRACE
  uint64_t tr[6] = {0, 0, 0, 0, 0, 0};
#endif
  for (;;) {
    if (wv == 0) {
      // wave 0 polls the whole request line: lanes 0-3 one 16-B piece each
      const volatile g_u32x4* src = (const volatile g_u32x4*)(box->line) + (lane & 3u);
      u32x4 v;
      bool stop = false;
      for (;;) {
        v = *src;
        const uint32_t tq = __builtin_amdgcn_readlane(v.x, 0);
        const bool ok = tq != last && tq == __builtin_amdgcn_readlane(v.x, 1) &&
                        tq == __builtin_amdgcn_readlane(v.x, 2) && tq == __builtin_amdgcn_readlane(v.x, 3);
        if (ok) break;
        if (static_cast<uint64_t>(wall_clock64()) - t0 > sa.idle_ticks) {
          stop = true;
          break;
        }
        __builtin_amdgcn_s_sleep(UGO_SVC_SLEEP);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
#ifdef UGO_SVC_TRACE
      tr[0] = wall_clock64();
#endif
      if (lane < 4u) {
        if (lane == 0 && stop) v.y = kSvcStop;
        line[lane] = v;
      }
      const uint32_t op = __builtin_amdgcn_readlane(v.y, 0), G = __builtin_amdgcn_readlane(v.z, 0);
      if (!stop && op == kSvcReconstruct) {
        if (lane == 0) {
          msk[0] = static_cast<uint64_t>(__builtin_amdgcn_readlane(v.y, 3)) << 32 | __builtin_amdgcn_readlane(v.w, 2);
          msk[1] = static_cast<uint64_t>(__builtin_amdgcn_readlane(v.w, 3)) << 32 | __builtin_amdgcn_readlane(v.z, 3);
        }
        if (lane >= 2u && lane < min(G, static_cast<uint32_t>(kSvcMaxGroups)))  // groups 2+: one more load
          msk[lane] = *(const volatile __attribute__((address_space(1))) uint64_t*)(&box->present[lane]);
      }
    }
    __syncthreads();
#ifdef UGO_SVC_TRACE
    tr[1] = wall_clock64();
#endif
    const uint32_t* rq = reinterpret_cast<const uint32_t*>(line);
    const uint32_t sq = rq[0], op = rq[1];
    if (op != kSvcEncode && op != kSvcReconstruct) break;
    const uint32_t G = min(rq[2], static_cast<uint32_t>(kSvcMaxGroups)), S = rq[3];
    uint8_t* base = reinterpret_cast<uint8_t*>(static_cast<uint64_t>(rq[6]) << 32 | rq[5]);
    const uint64_t pitch = static_cast<uint64_t>(rq[10]) << 32 | rq[9];
    const bool recon = op == kSvcReconstruct;
    const uint32_t data_only = recon && (rq[7] & 1u);
    if (sa.stall_ticks) {  // tests only: a slow block, to drive the host's watchdog
      const uint64_t ts = wall_clock64();
      while (static_cast<uint64_t>(wall_clock64()) - ts < sa.stall_ticks) __builtin_amdgcn_s_sleep(127);
    }
    if (recon) {  // this request's descriptors: one slot per group, a wave each
      for (uint32_t g = wv; g < G; g += kSvcThreads / 64u) {
        svc_copy_desc(L, g, a.desc + (msk[g] & a.nmask) * a.desc_stride, dwords, lane, 64u);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        svc_expand(L, g, a, lane, 64u);
      }
      __syncthreads();
    }
    const uint32_t chunks = (S + 15u) / 16u, cpad = (chunks + 63u) & ~63u;
    // A one-group request (ugo's per-group calls: 1470-B rows, 2 slices of 64
    // chunks) would leave 6 of the 8 waves idle while each busy wave folds
    // every output -- the fold was half the device time (tools/svc_trace.cpp).
    // Instead all waves load the survivors' (row, slice) pieces into LDS, then
    // each wave folds ONE output of one slice.
    constexpr uint32_t kWaves = kSvcThreads / 64u;
    // (with one output the fold is short and the staging would only add its
    // LDS round trip: 7.7 vs 7.2 us per 1-loss Reconstruct, so e >= 2 only)
    bool one = false;
    if (G == 1u && cpad <= 128u) {
      const uint32_t hdr = __builtin_amdgcn_readfirstlane(L.desc[recon ? 0u : ENC][0]);
      const uint32_t e = (hdr >> 16) & 0xffu ? 0u : (data_only ? ((hdr >> 8) & 0xffu) : (hdr & 0xffu));
      one = e >= 2u;
    }
    if (one) {
      const uint32_t slices = cpad / 64u;
      const uint32_t slot = recon ? 0u : ENC;
      const uint32_t* dw = L.desc[slot];
      const uint32_t hdr = __builtin_amdgcn_readfirstlane(dw[0]);
      const uint32_t e = data_only ? ((hdr >> 8) & 0xffu) : (hdr & 0xffu);  // status 0: e >= 2 above
      if (recon && threadIdx.x == 0) *(g_u8*)(&box->status[0]) = 0;
      {  // block-uniform
        // every (row, slice) piece by one wave; a wave's pieces all in flight at once
        constexpr uint32_t kPer = (2u * DMAX + kWaves - 1u) / kWaves;
        V4 v[kPer];
#pragma unroll
        for (uint32_t j = 0; j < kPer; ++j) {
          const uint32_t rs = wv + j * kWaves, k = rs / slices, sl = rs - k * slices, c = sl * 64u + lane;
          v[j] = V4{{0u, 0u, 0u, 0u}};
          if (rs < a.d * slices && c < chunks) {
            const uint32_t r = (__builtin_amdgcn_readfirstlane(dw[1u + (k >> 2)]) >> (8u * (k & 3u))) & 0xffu;
            v[j] = gload16(base + static_cast<uint64_t>(c) * 16u + static_cast<uint64_t>(r) * pitch);
          }
        }
#pragma unroll
        for (uint32_t j = 0; j < kPer; ++j) {
          const uint32_t rs = wv + j * kWaves, k = rs / slices, sl = rs - k * slices;
          if (rs < a.d * slices) L.rows[k][sl * 64u + lane] = u32x4{v[j].v[0], v[j].v[1], v[j].v[2], v[j].v[3]};
        }
        __syncthreads();
#ifdef UGO_SVC_TRACE
        tr[2] = wall_clock64();
#endif
        const uint32_t sl = wv >> 2, osel = wv & 3u;
        if (sl < slices && osel < e) {
          const uint32_t c = sl * 64u + lane;
          V4 x[DMAX];
#pragma unroll
          for (int k = 0; k < DMAX; ++k) {
            x[k] = V4{{0u, 0u, 0u, 0u}};
            if (k < static_cast<int>(a.d)) {
              const u32x4 v = L.rows[k][c];
              x[k] = V4{{v.x, v.y, v.z, v.w}};
            }
          }
          V4 y1 = V4{{0u, 0u, 0u, 0u}};
#pragma unroll
          for (int k = 0; k < DMAX; k += 2) {
            if (k >= static_cast<int>(a.d)) continue;
            uint32_t s0[4], s1[4], s2[4], r0[4], r1[4], r2[4];
            p_sel(x[k], s0, s1, s2);
            p_sel(x[k + 1], r0, r1, r2);
            const uint32_t* t = L.t[slot][osel][k];
            const uint32_t* u = L.t[slot][osel][k + 1];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              uint32_t y = xor3(y1.v[j], perm(t[1], t[0], s0[j]), perm(t[3], t[2], s1[j]));
              y = xor3(y, perm(0u, t[4], s2[j]), perm(u[1], u[0], r0[j]));
              y1.v[j] = xor3(y, perm(u[3], u[2], r1[j]), perm(0u, u[4], r2[j]));
            }
          }
          const uint32_t orows = __builtin_amdgcn_readfirstlane(dw[(4u + a.dpad) / 4u]);
          if (c < chunks)
            gstore16(base + static_cast<uint64_t>(c) * 16u + static_cast<uint64_t>((orows >> (8u * osel)) & 0xffu) * pitch,
                     y1, S - c * 16u);
        }
      }
    }
    // groups wave-aligned: wave w takes 64 chunks of one group at a time
    for (uint32_t w0 = wv * 64u; !one && w0 < G * cpad; w0 += kSvcThreads) {
      const uint32_t g = w0 / cpad;
      const uint32_t c = w0 - g * cpad + lane;
      const uint32_t slot = recon ? g : ENC;
      const uint32_t* dw = L.desc[slot];
      const uint32_t hdr = __builtin_amdgcn_readfirstlane(dw[0]);
      const uint32_t st = (hdr >> 16) & 0xffu;
      const uint32_t e = st ? 0u : (data_only ? ((hdr >> 8) & 0xffu) : (hdr & 0xffu));
      if (recon && c == 0) *(g_u8*)(&box->status[g]) = static_cast<uint8_t>(st);
      if (e == 0) continue;
      uint8_t* gp = base + static_cast<uint64_t>(g) * a.n * pitch + static_cast<uint64_t>(c) * 16u;
      V4 x[DMAX];
#pragma unroll
      for (int k = 0; k < DMAX; ++k) {
        x[k] = V4{{0u, 0u, 0u, 0u}};
        const uint32_t r = (__builtin_amdgcn_readfirstlane(dw[1 + (k >> 2)]) >> (8 * (k & 3))) & 0xffu;
        if (k < static_cast<int>(a.d) && c < chunks) x[k] = gload16(gp + static_cast<uint64_t>(r) * pitch);
      }
      const uint32_t orows = __builtin_amdgcn_readfirstlane(dw[(4u + a.dpad) / 4u]);
      V4 acc[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i] = V4{{0u, 0u, 0u, 0u}};
#pragma unroll
      for (int k = 0; k < DMAX; k += 2) {
        if (k >= static_cast<int>(a.d)) continue;
        uint32_t s0[4], s1[4], s2[4], r0[4], r1[4], r2[4];
        p_sel(x[k], s0, s1, s2);
        p_sel(x[k + 1], r0, r1, r2);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (i >= static_cast<int>(e)) continue;
          const uint32_t* t = L.t[slot][i][k];
          const uint32_t* u = L.t[slot][i][k + 1];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            uint32_t y = xor3(acc[i].v[j], perm(t[1], t[0], s0[j]), perm(t[3], t[2], s1[j]));
            y = xor3(y, perm(0u, t[4], s2[j]), perm(u[1], u[0], r0[j]));
            acc[i].v[j] = xor3(y, perm(u[3], u[2], r1[j]), perm(0u, u[4], r2[j]));
          }
        }
      }
      if (c < chunks) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (i >= static_cast<int>(e)) continue;
          const uint32_t r = (orows >> (8 * i)) & 0xffu;
          gstore16(gp + static_cast<uint64_t>(r) * pitch, acc[i], S - c * 16u);
        }
      }
    }
#ifdef UGO_SVC_TRACE
    tr[3] = wall_clock64();
#endif
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores have left
#ifdef UGO_SVC_TRACE
    tr[4] = wall_clock64();
#endif
    __syncthreads();
#ifdef UGO_SVC_TRACE
    tr[5] = wall_clock64();
    if (threadIdx.x == 0)
      for (int k = 0; k < 6; ++k) *(volatile __attribute__((address_space(1))) uint64_t*)(&box->trace[k]) = tr[k];
#endif
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __hip_atomic_store(&box->done, sq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    last = sq;
    t0 = wall_clock64();
  }
  if (threadIdx.x == 0) __hip_atomic_store(&box->alive, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Streaming form of k_apply_p for wide codes ((32,8) jumbo: d up to 255,
// e <= EMAX outputs): inputs are not held -- a 4-deep ring of survivor
// chunks is loaded ahead while the current pair is folded into EMAX live
// accumulators -- so registers hold 4*EMAX accumulator dwords plus the ring,
// independent of d (vs k_apply's d-sized input block and masked Horner).
template <int EMAX, int MODE, int NT, int TSEL = 1, int RING = 4>
__global__ __launch_bounds__(256) void k_apply_q(Batch a) {
  static_assert(RING % 2 == 0, "inputs are consumed in pairs");
  const uint32_t wfirst = blockIdx.x * 256u + (__builtin_amdgcn_readfirstlane(threadIdx.x) & ~63u);
  const uint32_t item = blockIdx.x * 256u + threadIdx.x;
  if (wfirst >= a.items) return;
  const uint32_t wlast = min(wfirst + 63u, a.items - 1u);
  const uint32_t gA = wfirst / a.chunks;
  const uint32_t gB = wlast / a.chunks;
  const uint8_t* dA = desc_for<MODE>(a, a.g0 + gA);
  const uint8_t* dB = desc_for<MODE>(a, a.g0 + gB);
  const uint32_t hA = ld32(dA), hB = ld32(dB);
  const uint32_t eA = ((hA >> 16) & 0xffu) ? 0u : (a.data_only ? ((hA >> 8) & 0xffu) : (hA & 0xffu));
  const uint32_t eB = ((hB >> 16) & 0xffu) ? 0u : (a.data_only ? ((hB >> 8) & 0xffu) : (hB & 0xffu));
  const uint32_t emax = max(eA, eB);
  if (item >= a.items) return;
  const uint32_t gl = item / a.chunks;
  const bool inB = gl != gA;
  const uint32_t c = item - gl * a.chunks;
  const uint64_t g = a.g0 + gl;
  const uint32_t st = ((inB ? hB : hA) >> 16) & 0xffu;
  const bool wst = MODE != 0 && a.status != nullptr && c == 0;
  const uint32_t e = inB ? eB : eA;
  if (e == 0) {
    if (wst) a.status[g] = static_cast<int8_t>(st);
    return;
  }
  uint32_t mB;
  asm("v_mov_b32 %0, %1" : "=v"(mB) : "v"(inB ? ~0u : 0u));
  // wave-uniform descriptor (always, in MODE 0: one descriptor for the batch,
  // so the two-group table pick is compiled out and the table words stay SGPRs)
  const uint8_t* dS = (MODE == 0 || dA == dB) ? dA : nullptr;
  uint8_t* gp = a.base + g * a.gstride + static_cast<uint64_t>(c) * 16u;
  const uint32_t nb = a.S - c * 16u;
  auto row_of = [&](uint32_t k) -> uint32_t {
    const uint32_t wa = ld32(dA + 4 + (k & ~3u)), wb = ld32(dB + 4 + (k & ~3u));
    return ((inB ? wb : wa) >> (8 * (k & 3u))) & 0xffu;
  };
  auto load_in = [&](uint32_t k) -> V4 {
    if (k >= a.d) return V4{{0u, 0u, 0u, 0u}};
    return load16<NT>(gp + static_cast<uint64_t>(row_of(k)) * a.rstride);
  };
  V4 acc[EMAX];
#pragma unroll
  for (int i = 0; i < EMAX; ++i) acc[i] = V4{{0u, 0u, 0u, 0u}};
  V4 ring[RING];
#pragma unroll
  for (int j = 0; j < RING; ++j) ring[j] = load_in(j);
  const uint32_t cbase = 4 + a.dpad + a.epad;
  for (uint32_t k0 = 0; k0 < a.d; k0 += RING) {
#pragma unroll
    for (int j = 0; j < RING; j += 2) {
      const uint32_t k = k0 + j;
      uint32_t s0[4], s1[4], s2[4], r0[4], r1[4], r2[4];
      p_sel(ring[j], s0, s1, s2);
      p_sel(ring[j + 1], r0, r1, r2);
      ring[j] = load_in(k + RING);
      ring[j + 1] = load_in(k + RING + 1);
#pragma unroll
      for (int i = 0; i < EMAX; ++i) {
        if (i >= static_cast<int>(emax)) continue;
        const uint32_t off = cbase + i * a.dpad + (k & ~3u);  // coefficient word of inputs k, k+1
        // byte of input k in that word (compile-time when the ring is a multiple of 4)
        const int kb = RING % 4 == 0 ? (j & 3) : static_cast<int>(k & 3u);
        uint32_t t[5], u[5];
        if (MODE == 0 || dS) {
          p_tables<0>(t, a, dS, dS, off, kb, 0u);
          p_tables<0>(u, a, dS, dS, off, kb + 1, 0u);
        } else {
          p_tables<TSEL>(t, a, dA, dB, off, kb, mB);
          p_tables<TSEL>(u, a, dA, dB, off, kb + 1, mB);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          uint32_t y = xor3(acc[i].v[q], perm(t[1], t[0], s0[q]), perm(t[3], t[2], s1[q]));
          y = xor3(y, perm(0u, t[4], s2[q]), perm(u[1], u[0], r0[q]));
          acc[i].v[q] = xor3(y, perm(u[3], u[2], r1[q]), perm(0u, u[4], r2[q]));
        }
      }
    }
  }
  constexpr int NO = (EMAX + 3) / 4;
  uint32_t orw[NO];
#pragma unroll
  for (int w = 0; w < NO; ++w) {
    const uint32_t oa = ld32(dA + 4 + a.dpad + 4 * w), ob = ld32(dB + 4 + a.dpad + 4 * w);
    orw[w] = inB ? ob : oa;
  }
#pragma unroll
  for (int i = 0; i < EMAX; ++i) {
    if (i >= static_cast<int>(e)) continue;
    const uint32_t r = (orw[i >> 2] >> (8 * (i & 3))) & 0xffu;
    store16<NT>(out_row(a, gp, g, c * 16u, r, i), acc[i], nb);
  }
  if (wst) a.status[g] = 0;
}

// Wave-aligned form of k_apply_q, for rows whose chunk count is just under a
// multiple of 64 ((32,8) x 9000: 563 of 576 lanes busy): every group starts
// at a wave boundary (item = group * cpad + chunk, cpad = chunks rounded up to
// 64; the launcher sets items = groups * cpad), so a wave never spans two
// groups.  Its descriptor is wave-uniform, the table words stay SGPRs and each
// v_perm reads its low word from the constant bus: 4 VGPR copies per product
// pair instead of the 10 of k_apply_q, whose merged uniform / two-group paths
// make every table word a VGPR.  A 2-deep input ring keeps it at 79 VGPRs (6
// waves/SIMD; the 4-deep ring takes 113 and 4 waves): 533.5 against 550.4 us
// for the jumbo reconstruct (profiles/r2/jvariants_qa_ring2.jsonl).  Lanes
// past the row's end load chunk 0 and store nothing.
// PASSES: more than EMAX outputs (wide-parity codes past d = 32) are folded
// EMAX at a time, the inputs re-read per pass (L2-resident by then).
template <int EMAX, int MODE, int NT, int RING = 2, int WPE = 1, bool PASSES = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_apply_qa(Batch a) {
  static_assert(RING % 2 == 0, "inputs are consumed in pairs");
  const uint32_t cpad = (a.chunks + 63u) & ~63u;
  const uint32_t wfirst = blockIdx.x * 256u + (__builtin_amdgcn_readfirstlane(threadIdx.x) & ~63u);
  if (wfirst >= a.items) return;  // a.items = groups * cpad here
  const uint32_t gl = wfirst / cpad;  // wave-uniform
  const uint64_t g = a.g0 + gl;
  const uint8_t* dA = desc_for<MODE>(a, g);
  const uint32_t hA = ld32(dA);
  const uint32_t st = (hA >> 16) & 0xffu;
  const uint32_t e = st ? 0u : (a.data_only ? ((hA >> 8) & 0xffu) : (hA & 0xffu));
  const uint32_t c = blockIdx.x * 256u + threadIdx.x - gl * cpad;
  const bool live = c < a.chunks;
  const bool wst = MODE != 0 && a.status != nullptr && c == 0;
  if (e == 0) {  // wave-uniform
    if (wst) a.status[g] = static_cast<int8_t>(st);
    return;
  }
  const uint32_t coff = live ? c * 16u : 0u;
  uint8_t* gp = a.base + g * a.gstride + coff;
  auto load_in = [&](uint32_t k) -> V4 {
    if (k >= a.d) return V4{{0u, 0u, 0u, 0u}};
    const uint32_t r = (ldw<PASSES>(dA + 4 + (k & ~3u)) >> (8 * (k & 3u))) & 0xffu;
    return load16<NT>(gp + static_cast<uint64_t>(r) * a.rstride);
  };
  const uint32_t cbase = 4 + a.dpad + a.epad;
  // outputs [ob, ob + en) of this pass (one pass of all e outputs unless PASSES)
  auto run = [&](uint32_t ob, uint32_t en) {
    V4 acc[EMAX];
#pragma unroll
    for (int i = 0; i < EMAX; ++i) acc[i] = V4{{0u, 0u, 0u, 0u}};
    V4 ring[RING];
#pragma unroll
    for (int j = 0; j < RING; ++j) ring[j] = load_in(j);
    for (uint32_t k0 = 0; k0 < a.d; k0 += RING) {
#pragma unroll
      for (int j = 0; j < RING; j += 2) {
        const uint32_t k = k0 + j;
        uint32_t s0[4], s1[4], s2[4], r0[4], r1[4], r2[4];
        p_sel(ring[j], s0, s1, s2);
        p_sel(ring[j + 1], r0, r1, r2);
        ring[j] = load_in(k + RING);
        ring[j + 1] = load_in(k + RING + 1);
#pragma unroll
        for (int i = 0; i < EMAX; ++i) {
          if (i >= static_cast<int>(en)) continue;
          const uint32_t off = cbase + (ob + i) * a.dpad + (k & ~3u);  // coefficient word of inputs k, k+1
          const int kb = RING % 4 == 0 ? (j & 3) : static_cast<int>(k & 3u);
          uint32_t t[5], u[5];
          if constexpr (PASSES) {  // tables read after the previous pass's stores
            p_tables_u<true>(t, a, dA, off, kb);
            p_tables_u<true>(u, a, dA, off, kb + 1);
          } else {
            p_tables<0>(t, a, dA, dA, off, kb, 0u);
            p_tables<0>(u, a, dA, dA, off, kb + 1, 0u);
          }
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            uint32_t y = xor3(acc[i].v[q], perm(t[1], t[0], s0[q]), perm(t[3], t[2], s1[q]));
            y = xor3(y, perm(0u, t[4], s2[q]), perm(u[1], u[0], r0[q]));
            acc[i].v[q] = xor3(y, perm(u[3], u[2], r1[q]), perm(0u, u[4], r2[q]));
          }
        }
      }
    }
    if (live) {
      const uint32_t nb = a.S - coff;
      constexpr int NO = (EMAX + 3) / 4;
      uint32_t orw[NO];
#pragma unroll
      for (int w = 0; w < NO; ++w) orw[w] = ldw<PASSES>(dA + 4 + a.dpad + ob + 4 * w);  // ob % 4 == 0
#pragma unroll
      for (int i = 0; i < EMAX; ++i) {
        if (i >= static_cast<int>(en)) continue;
        const uint32_t r = (orw[i >> 2] >> (8 * (i & 3))) & 0xffu;
        store16<NT>(out_row(a, gp, g, coff, r, ob + i), acc[i], nb);
      }
    }
  };
  if constexpr (PASSES) {
    for (uint32_t ob = 0; ob < e; ob += EMAX) run(ob, min(e - ob, static_cast<uint32_t>(EMAX)));
  } else {
    run(0u, e);
  }
  if (wst) a.status[g] = 0;
}

// 64-bit wave-uniform value into SGPRs.
__device__ __forceinline__ uint64_t rfl64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

// k_apply_qa with its per-product overhead cut (round 3, the jumbo
// reconstruct).  The ISA of k_apply_qa showed three VALU costs beside the
// 3 v_perm + 1.5 v_bitop3 per product dword:
//   OPT & 1: the descriptor pointer came out of a VALU division (group =
//            wave offset / padded row), lived in VGPRs, and every scalar
//            coefficient load paid two v_readfirstlane: now made SGPR once;
//   OPT & 2: each input load computed its 64-bit address per lane (v_mov +
//            v_mad_u64_u32 + v_add): now the row base is uniform (SGPRs) and
//            the lane adds a 32-bit offset (the global saddr form);
//   OPT & 4: the 2-deep input ring was rotated by 8 v_mov per pair: now the
//            loop is unrolled over two pairs, each loaded into its own
//            registers.
template <int EMAX, int MODE, int NT, int OPT = 7, int WPE = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_apply_qb(Batch a) {
  const uint32_t cpad = (a.chunks + 63u) & ~63u;
  // OPT & 32 (grid a multiple of 8): XCD-contiguous blocks -- the hardware
  // deals blocks to the 8 XCDs round robin; block b works on tile
  // (b % 8) * (grid / 8) + b / 8, so each XCD sweeps one contiguous eighth
  // and the 2-3 blocks of one group read its descriptor through one L2
  uint32_t bid = blockIdx.x;
  if constexpr (OPT & 32) bid = (blockIdx.x & 7u) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  const uint32_t wfirst = bid * 256u + (__builtin_amdgcn_readfirstlane(threadIdx.x) & ~63u);
  if (wfirst >= a.items) return;  // a.items = groups * cpad here
  const uint32_t gl = (OPT & 1) ? __builtin_amdgcn_readfirstlane(wfirst / cpad) : wfirst / cpad;
  const uint64_t g = a.g0 + gl;
  const uint8_t* dA = desc_for<MODE>(a, g);
  // OPT & 1: descriptor words and coefficient tables through the constant
  // address space from an SGPR base (a plain pointer made uniform by
  // readfirstlane turns them into flat / per-lane vector loads)
  const uint64_t dU = (OPT & 1) ? rfl64(reinterpret_cast<uint64_t>(dA)) : 0;
  auto dword = [&](uint32_t off) -> uint32_t {
    if constexpr (OPT & 1)
      return *(ctab_t)(dU + off);
    else
      return ld32(dA + off);
  };
  const uint32_t hA = dword(0);
  const uint32_t st = (hA >> 16) & 0xffu;
  const uint32_t e = st ? 0u : (a.data_only ? ((hA >> 8) & 0xffu) : (hA & 0xffu));
  const uint32_t c = bid * 256u + threadIdx.x - gl * cpad;
  const bool live = c < a.chunks;
  const bool wst = MODE != 0 && a.status != nullptr && c == 0;
  if (e == 0) {  // wave-uniform
    if (wst) a.status[g] = static_cast<int8_t>(st);
    return;
  }
  const uint32_t coff = live ? c * 16u : 0u;
  const uint8_t* gbase = a.base + g * a.gstride;  // wave-uniform
  auto load_in = [&](uint32_t k) -> V4 {
    if (k >= a.d) return V4{{0u, 0u, 0u, 0u}};
    const uint32_t r = (dword(4 + (k & ~3u)) >> (8 * (k & 3u))) & 0xffu;
    if constexpr (OPT & 2) {
      const uint8_t* rb = gbase + static_cast<uint64_t>(r) * a.rstride;  // SGPRs
      uint32_t co = coff;
      asm("" : "+v"(co));  // opaque per load: gbase + coff is not hoisted into a 64-bit VGPR pair
      return load16<NT>(rb + co);
    } else {
      return load16<NT>(gbase + coff + static_cast<uint64_t>(r) * a.rstride);
    }
  };
  auto tables = [&](uint32_t* t, uint32_t off, int kb) {
    const uint32_t cf = (dword(off) >> (8 * (kb & 3))) & 0xffu;
    if constexpr (OPT & 1) {
      const ctab_t tA = (ctab_t)(a.mult) + 8u * cf;
#pragma unroll
      for (int q = 0; q < 5; ++q) t[q] = tA[q];
    } else {
      const uint32_t* tA = a.mult + 8u * cf;
#pragma unroll
      for (int q = 0; q < 5; ++q) t[q] = tA[q];
    }
  };
  const uint32_t cbase = 4 + a.dpad + a.epad;
  V4 acc[EMAX];
#pragma unroll
  for (int i = 0; i < EMAX; ++i) acc[i] = V4{{0u, 0u, 0u, 0u}};
  // fold the pair (k, k+1) whose selectors are s, r into the accumulators
  // (OPT & 8, A/B only: the memory pattern alone -- inputs XORed, no products)
  auto fold = [&](uint32_t k, const uint32_t* s0, const uint32_t* s1, const uint32_t* s2, const uint32_t* r0,
                  const uint32_t* r1, const uint32_t* r2, int kb) {
    if constexpr (OPT & 8) {
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[0].v[q] = xor3(acc[0].v[q], s0[q], r0[q]);
#pragma unroll
      for (int i = 1; i < EMAX; ++i) acc[i] = acc[0];
      return;
    }
#pragma unroll
    for (int i = 0; i < EMAX; ++i) {
      if (i >= static_cast<int>(e)) continue;
      const uint32_t off = cbase + i * a.dpad + (k & ~3u);  // coefficient word of inputs k, k+1
      uint32_t t[5], u[5];
      tables(t, off, kb);
      tables(u, off, kb + 1);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t y = xor3(acc[i].v[q], perm(t[1], t[0], s0[q]), perm(t[3], t[2], s1[q]));
        y = xor3(y, perm(0u, t[4], s2[q]), perm(u[1], u[0], r0[q]));
        acc[i].v[q] = xor3(y, perm(u[3], u[2], r1[q]), perm(0u, u[4], r2[q]));
      }
    }
  };
  if constexpr (OPT & 4) {
    // k0 % 4 == 0: pair A = inputs k0, k0+1 (coefficient bytes 0, 1 of the word),
    // pair B = k0+2, k0+3 (bytes 2, 3); A's next pair is loaded after A's selectors
    V4 a0 = load_in(0), a1 = load_in(1);
    for (uint32_t k0 = 0; k0 < a.d; k0 += 4) {
      uint32_t s0[4], s1[4], s2[4], r0[4], r1[4], r2[4];
      p_sel(a0, s0, s1, s2);
      p_sel(a1, r0, r1, r2);
      const V4 b0 = load_in(k0 + 2), b1 = load_in(k0 + 3);
      fold(k0, s0, s1, s2, r0, r1, r2, 0);
      p_sel(b0, s0, s1, s2);
      p_sel(b1, r0, r1, r2);
      a0 = load_in(k0 + 4);
      a1 = load_in(k0 + 5);
      fold(k0 + 2, s0, s1, s2, r0, r1, r2, 2);
    }
  } else {
    V4 ring[2] = {load_in(0), load_in(1)};
    for (uint32_t k = 0; k < a.d; k += 2) {
      uint32_t s0[4], s1[4], s2[4], r0[4], r1[4], r2[4];
      p_sel(ring[0], s0, s1, s2);
      p_sel(ring[1], r0, r1, r2);
      ring[0] = load_in(k + 2);
      ring[1] = load_in(k + 3);
      fold(k, s0, s1, s2, r0, r1, r2, static_cast<int>(k & 3u));
    }
  }
  if (live) {
    const uint32_t nb = a.S - coff;
    constexpr int NO = (EMAX + 3) / 4;
    uint32_t orw[NO];
#pragma unroll
    for (int w = 0; w < NO; ++w) orw[w] = dword(4 + a.dpad + 4 * w);
    uint8_t* gp = const_cast<uint8_t*>(gbase) + coff;
#pragma unroll
    for (int i = 0; i < EMAX; ++i) {
      if (i >= static_cast<int>(e)) continue;
      const uint32_t r = (orw[i >> 2] >> (8 * (i & 3))) & 0xffu;
      store16<NT>(out_row(a, gp, g, coff, r, i), acc[i], nb);
    }
  }
  if (wst) a.status[g] = 0;
}

// generic: any alignment / stride / d (<= 255); 4 columns per lane, byte I/O
__device__ __forceinline__ uint32_t gfmul_var(uint32_t cbyte, uint32_t x) {
  uint32_t t = 0;
#pragma unroll
  for (int b = 7; b >= 0; --b) {
    t = xt1(t);
    const uint32_t m = static_cast<uint32_t>(-static_cast<int32_t>((cbyte >> b) & 1u));
    t = xor_and(t, x, m);
  }
  return t;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_apply_bytes(Batch a) {
  const uint32_t item = blockIdx.x * 256u + threadIdx.x;
  if (item >= a.items) return;
  const uint32_t gl = item / a.chunks;  // chunks = ceil(S / 4) here
  const uint32_t c = item - gl * a.chunks;
  const uint64_t g = a.g0 + gl;
  const uint8_t* desc = desc_for<MODE>(a, g);
  const uint32_t hdr = ld32(desc);
  const uint32_t st = (hdr >> 16) & 0xffu;
  if (MODE != 0 && a.status != nullptr && c == 0) a.status[g] = static_cast<int8_t>(st);
  const uint32_t e = a.data_only ? ((hdr >> 8) & 0xffu) : (hdr & 0xffu);
  if (st != 0 || e == 0) return;
  uint8_t* gp = a.base + g * a.gstride + static_cast<uint64_t>(c) * 4u;
  const uint32_t nb = min(4u, a.S - c * 4u);
  const uint8_t* irow = desc + 4;
  const uint8_t* orow = desc + 4 + a.dpad;
  const uint8_t* coef = orow + a.epad;
  for (uint32_t i = 0; i < e; ++i) {
    uint32_t acc = 0;
    for (uint32_t k = 0; k < a.d; ++k) {
      const uint8_t* src = gp + static_cast<uint64_t>(irow[k]) * a.rstride;
      uint32_t x = 0;
      for (uint32_t j = 0; j < nb; ++j) x |= static_cast<uint32_t>(src[j]) << (8 * j);
      acc ^= gfmul_var(coef[i * a.dpad + k], x);
    }
    uint8_t* dst = out_row(a, gp, g, c * 4u, orow[i], i);
    for (uint32_t j = 0; j < nb; ++j) dst[j] = static_cast<uint8_t>(acc >> (8 * j));
  }
}

// ------------------------------------------------------------ k_apply_rows
// Reconstruct from a row-pointer table (ugo_fec_reconstruct_rows): row r of
// group g is rows[g*(d+p) + r], a device address anywhere -- typically a
// pooled packet buffer in pinned host memory, read over PCIe in place (the
// FEC object's batched recovery: no copy of the survivors into a batch).
// One 16-byte chunk per thread; survivors in blocks of 16 (their loads issued
// together: over PCIe each load is microseconds of latency), products by the
// v_perm split tables; outputs folded 8 per pass; recovered rows go to the
// caller's output batch, output i = the i-th erased row (ascending).  A group
// whose survivor pointers are not 16-B aligned gets UGO_FEC_ERR_INVALID_ARG
// and is not touched.  Latency / PCIe-bound: batches of tens of groups.
typedef const __attribute__((address_space(1))) u32x4* gptr16_t;

// One 16-byte chunk of a row (rows are readable in whole 16-B granules: the
// reconstruct_rows contract), through a global-space pointer (a generic one
// would make it a flat load).
__device__ __forceinline__ V4 load_row16(uint64_t p) {
  const u32x4 v = *(gptr16_t)(p);
  return V4{{v.x, v.y, v.z, v.w}};
}

// Wave-aligned groups (item = group * cpad + chunk, cpad = chunks rounded up to
// 64, as k_apply_qa): everything but the row bytes is wave-uniform and read
// with scalar loads -- descriptor, row pointers, coefficient tables.  The
// kernel is latency-bound (tens of groups per launch, rows over PCIe), so its
// code is kept small: outputs in a rolled loop, one accumulator, the
// survivors' selectors recomputed per output.  Fully unrolled over 16 inputs
// x 8 outputs (10 K instructions) it took 14 us for ONE group even with
// every buffer in HBM: cold instruction fetch, not memory (tools/rows_probe.py,
// profiles/r3/rows_probe.jsonl).
typedef const __attribute__((address_space(4))) uint64_t* ctab64_t;

// acc ^= sum over the block's inputs j of c(i, k0 + j) * x[j]
template <int NB>
__device__ __forceinline__ void rows_fold(V4& acc, const V4* x, const Batch& a, uint64_t dU, uint32_t coff_i,
                                          uint32_t k0) {
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    if (k0 + j >= a.d) continue;
    uint32_t s0[4], s1[4], s2[4];
    p_sel(x[j], s0, s1, s2);
    const uint32_t o = coff_i + k0 + j;
    const uint32_t cf = (*(ctab_t)(dU + (o & ~3u)) >> (8u * (o & 3u))) & 0xffu;
    const ctab_t t = (ctab_t)(a.mult) + 8u * cf;
#pragma unroll
    for (int w = 0; w < 4; ++w)
      acc.v[w] = xor3(acc.v[w], perm(t[1], t[0], s0[w]), perm(t[3], t[2], s1[w])) ^ perm(0u, t[4], s2[w]);
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void k_apply_rows(Batch a) {
  constexpr int NB = 16;  // inputs per block (d <= 16: one block, loaded once)
  const uint32_t cpad = (a.chunks + 63u) & ~63u;
  const uint32_t wfirst = blockIdx.x * 256u + (__builtin_amdgcn_readfirstlane(threadIdx.x) & ~63u);
  if (wfirst >= a.items) return;  // a.items = groups * cpad
  const uint32_t gl = __builtin_amdgcn_readfirstlane(wfirst / cpad);
  const uint64_t g = a.g0 + gl;
  const uint64_t dU = rfl64(reinterpret_cast<uint64_t>(desc_for<MODE>(a, g)));
  auto dbyte = [&](uint32_t off) -> uint32_t { return (*(ctab_t)(dU + (off & ~3u)) >> (8u * (off & 3u))) & 0xffu; };
  const uint32_t hdr = *(ctab_t)(dU);
  const uint32_t st = (hdr >> 16) & 0xffu;
  const uint32_t e = a.data_only ? ((hdr >> 8) & 0xffu) : (hdr & 0xffu);
  const uint32_t c = blockIdx.x * 256u + threadIdx.x - gl * cpad;
  const bool live = c < a.chunks;
  const bool wst = a.status != nullptr && c == 0;
  if (st != 0 || e == 0) {  // wave-uniform
    if (wst) a.status[g] = static_cast<int8_t>(st);
    return;
  }
  const ctab64_t rp = (ctab64_t)(a.rows + g * a.n);  // the group's row pointers (scalar loads)
  // every survivor pointer checked before anything is read or written: a null
  // or misaligned one fails the group (UGO_FEC_ERR_INVALID_ARG, 6), untouched
  uint64_t bad = 0;
  for (uint32_t k = 0; k < a.d; ++k) {
    const uint64_t q = rp[dbyte(4 + k)];
    bad |= (q & 15u) | (q == 0);
  }
  if (bad) {
    if (wst) a.status[g] = 6;
    return;
  }
  const uint32_t cbase = 4 + a.dpad + a.epad;
  const uint32_t off = live ? c * 16u : 0u;
  const uint32_t nb = live ? min(16u, a.S - off) : 16u;
  auto load_block = [&](V4* x, uint32_t k0) {  // the block's row loads, issued together
#pragma unroll
    for (int j = 0; j < NB; ++j)
      x[j] = (k0 + j < a.d) ? load_row16(rp[dbyte(4 + k0 + j)] + off) : V4{{0u, 0u, 0u, 0u}};
  };
  V4 x[NB];
  if (a.d <= static_cast<uint32_t>(NB)) load_block(x, 0);
  for (uint32_t i = 0; i < e; ++i) {
    V4 acc{{0u, 0u, 0u, 0u}};
    if (a.d <= static_cast<uint32_t>(NB)) {
      rows_fold<NB>(acc, x, a, dU, cbase + i * a.dpad, 0);
    } else {
      for (uint32_t k0 = 0; k0 < a.d; k0 += NB) {  // wide codes: the rows re-read per output
        load_block(x, k0);
        rows_fold<NB>(acc, x, a, dU, cbase + i * a.dpad, k0);
      }
    }
    if (live) store16<0>(a.out + g * a.ogstride + static_cast<uint64_t>(i) * a.orstride + off, acc, nb);
  }
  if (wst) a.status[g] = 0;
}

// ------------------------------------------------------------- k_prepare
// One 64-lane wave per group builds that group's decode descriptor:
// survivors = first d present rows (index order), A = M[survivors], Gauss-Jordan
// over GF(2^8) in LDS, then coefficient rows: Dinv[r] for an erased data row r,
// M[r] * Dinv for an erased parity row r.  d + p <= 64, so d <= 63 rows fit
// the wave's lanes one row per lane.
// One wave per group.  The survivors are the first d present rows: the
// present data rows P (identity rows of M) then the first e_d present parity
// rows J, where e_d = number of erased data rows E.  So the d x d inverse
// reduces to the e_d x e_d block B = M[J][E]:
//     x_E = B^-1 (y_J + M[J][P] y_P)          (GF(2^8): minus is plus)
//   Dinv[E_l][pos(J_i)] = Binv[l][i],  Dinv[E_l][pos(P_m)] = sum_i Binv[l][i] M[J_i][P_m]
// and an erased parity row r gets M[r]·Dinv:
//   coef[pos(P_m)] = M[r][P_m] + sum_l M[r][E_l] Dinv[E_l][pos],  coef[pos(J_i)] = sum_l M[r][E_l] Binv[l][i]
// The same linear map as the full Gauss-Jordan of klauspost's Reconstruct
// (exact arithmetic), at e_d^3 + e_d^2 d instead of d^3 work.
//
// prep_wave is the body: ONE wave builds group g's descriptor at `desc`
// (global workspace for k_prepare, LDS for k_apply_gq) with its scratch in
// `s`.  It synchronises only its own lanes (wsync: a wave's LDS operations
// complete in order, so a code-motion barrier is enough), so one wave of a
// larger block can run it while the others do something else.
template <int NMD>
struct PrepSharedT {    // per block: staged once, read by every wave
  uint8_t ex[512];
  uint8_t lg[256];
  uint8_t M[NMD];       // the (d+p) x d encoding matrix, NMD >= (d+p) d
};
template <int EDM>
struct PrepWaveT {      // per wave (per group being built), EDM >= e_d
  uint8_t Ba[EDM * 2 * EDM];  // [B | I]
  uint8_t DE[EDM * 64];       // Dinv rows of the erased data rows, over survivor positions
  uint8_t fcol[32];     // log of column r of the pivot step (255 = zero)
  uint8_t lrow[64];     // log of pivot row r scaled by 1/pivot
  uint8_t surv[64], outr[64], Pl[64], El[64], Jl[64];
};
// Any code (e_d <= min(d, p) <= 32 since d + p <= 64), and the small tier
// k_prepare launches for codes with min(d, p) <= 8 and (d+p) d <= 2048 (the
// (32,8) jumbo): 7 KiB of LDS per block instead of 22.9, so LDS no longer
// caps the blocks per CU.
using PrepShared = PrepSharedT<64 * 64>;
using PrepWave = PrepWaveT<32>;
constexpr int kPrepSmallEdm = 8, kPrepSmallNmd = 2048, kPrepSmallWpe = 1;

// Branch-free product: the lookups always run (lg[0] is a valid byte), the
// select zeroes them, so a lane never diverges around an LDS read.
__device__ __forceinline__ uint32_t lmul(const uint8_t* lg, const uint8_t* ex, uint32_t a, uint32_t b) {
  const uint32_t t = ex[lg[a] + lg[b]];
  return (a && b) ? t : 0u;
}

// floor(x / w) for x < 2^11 and 1 <= w <= 64 as a multiply by rw =
// ceil(2^20 / w): the reciprocal's error, below x / 2^20 < 1/64, cannot carry
// a quotient past the next integer (the fraction of x / w is at most 1 - 1/w).
// The descriptor build's index splits would otherwise be ~20-instruction
// integer divisions, a third of its VALU work.
__device__ __forceinline__ uint32_t rcp_small(uint32_t w) { return ((1u << 20) + w - 1) / w; }
__device__ __forceinline__ uint32_t div_small(uint32_t x, uint32_t rw) { return (x * rw) >> 20; }

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Stage the GF tables and M into LDS with 16-B loads by threads [0, nthr):
// every later read of the descriptor build is an LDS read (global reads
// inside its dependent loops cost a full memory latency each under load).
// The caller synchronises before prep_wave reads them.
template <typename PS>
__device__ __forceinline__ void prep_stage(const Prep& a, PS& s, uint32_t tid, uint32_t nthr) {
  const uint32_t mb = a.n * a.d, m16 = mb / 16;
  for (uint32_t i = tid; i < 32 + 16 + m16; i += nthr) {
    const u32x4* src = i < 32 ? reinterpret_cast<const u32x4*>(a.gf_exp) + i
                     : i < 48 ? reinterpret_cast<const u32x4*>(a.gf_log) + (i - 32)
                              : reinterpret_cast<const u32x4*>(a.M) + (i - 48);
    u32x4* dst = i < 32 ? reinterpret_cast<u32x4*>(s.ex) + i
               : i < 48 ? reinterpret_cast<u32x4*>(s.lg) + (i - 32)
                        : reinterpret_cast<u32x4*>(s.M) + (i - 48);
    *dst = *src;
  }
  for (uint32_t i = m16 * 16 + tid; i < mb; i += nthr) s.M[i] = a.M[i];
}

template <typename DescPtr, typename PS, typename PW>
__device__ __forceinline__ void prep_wave(const Prep& a, uint64_t g, DescPtr desc, const PS& sh, PW& s,
                                          uint32_t lane) {
  const uint32_t d = a.d, n = a.n;
  const uint8_t* M = sh.M;
  const uint64_t mask = a.present[g] & a.nmask;
  const uint32_t np = __popcll(mask);
  if (np == n || np < d) {
    if (lane == 0) {
      const uint32_t st = np < d ? 3u : 0u;
      *reinterpret_cast<uint32_t*>(desc) = st << 16;
    }
    return;
  }
  const uint8_t* lg = sh.lg;
  const uint8_t* ex = sh.ex;
  const uint64_t dmask = (d >= 64) ? ~0ull : ((1ull << d) - 1);
  const uint64_t below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const uint32_t e = n - np;
  const uint32_t ed = __popcll(~mask & dmask);  // erased data rows
  const uint32_t npd = d - ed;                  // present data rows
  if (lane < n) {
    const bool present = (mask >> lane) & 1ull;
    if (lane < d) {
      if (present) s.Pl[__popcll(mask & dmask & below)] = static_cast<uint8_t>(lane);
      else s.El[__popcll(~mask & dmask & below)] = static_cast<uint8_t>(lane);
    } else if (present) {
      const uint32_t rank = __popcll(mask & ~dmask & below);
      if (rank < ed) s.Jl[rank] = static_cast<uint8_t>(lane);
    }
    if (!present) s.outr[__popcll(~mask & a.nmask & below)] = static_cast<uint8_t>(lane);
  }
  wsync();
  if (lane < d) s.surv[lane] = lane < npd ? s.Pl[lane] : s.Jl[lane - npd];
  // [B | I], B[i][l] = M[J_i][E_l]
  const uint32_t w = 2 * ed;
  const uint32_t rw = rcp_small(w ? w : 1u), rd = rcp_small(d), rdp = rcp_small(a.dpad);  // wave-uniform
  for (uint32_t idx = lane; idx < ed * w; idx += 64) {
    const uint32_t i = div_small(idx, rw), col = idx - i * w;
    s.Ba[idx] = col < ed ? M[s.Jl[i] * d + s.El[col]] : static_cast<uint8_t>(col - ed == i ? 1 : 0);
  }
  wsync();
  {
    // Log-domain pivot step, 4 dependent LDS round trips: (pivot, row r,
    // column r) -> their logs -> [store, sync] -> (row log, column log, entry)
    // -> exp.  Row r is scaled by 1/pivot inside the logs, so every entry of
    // the step is one product.  Pivots of an MDS code's B are never zero
    // (every leading block is a square submatrix of the parity rows); the
    // swap stays for safety.
    for (uint32_t r = 0; r < ed; ++r) {
      uint32_t piv = s.Ba[r * w + r];
      uint32_t x = lane < w ? s.Ba[r * w + lane] : 0u;
      uint32_t y = lane < ed ? s.Ba[lane * w + r] : 0u;
      if (piv == 0) {  // uniform
        const bool cand = lane > r && lane < ed && y != 0;
        const uint64_t bal = __ballot(cand);
        if (bal == 0) {
          if (lane == 0) *reinterpret_cast<uint32_t*>(desc) = 7u << 16;
          return;
        }
        const uint32_t b = __ffsll(static_cast<long long>(bal)) - 1;
        if (lane < w) {
          const uint8_t t = s.Ba[b * w + lane];
          s.Ba[b * w + lane] = static_cast<uint8_t>(x);
          s.Ba[r * w + lane] = t;
        }
        wsync();
        piv = s.Ba[r * w + r];
        x = lane < w ? s.Ba[r * w + lane] : 0u;
        y = lane < ed ? s.Ba[lane * w + r] : 0u;
      }
      const uint32_t pinv = 255u - sh.lg[piv];
      const uint32_t lx = lg[x], ly = lg[y];
      uint32_t t = lx + pinv;
      t = t >= 255u ? t - 255u : t;
      if (lane < w) s.lrow[lane] = static_cast<uint8_t>(x ? t : 255u);
      if (lane < ed) s.fcol[lane] = static_cast<uint8_t>(y ? ly : 255u);
      wsync();
#pragma unroll 2
      for (uint32_t idx = lane; idx < ed * w; idx += 64) {
        const uint32_t o = div_small(idx, rw), col = idx - o * w;
        const uint32_t lr = s.lrow[col], lc = s.fcol[o], cur = s.Ba[idx];
        const uint32_t pr = ex[lr + (o == r ? 0u : lc)];
        const uint32_t pz = (lr == 255u || lc == 255u) ? 0u : pr;
        s.Ba[idx] = static_cast<uint8_t>(o == r ? (lr == 255u ? 0u : pr) : cur ^ pz);
      }
      wsync();
    }
  }
  // Dinv rows of the erased data rows (Binv = Ba[:, ed:])
  for (uint32_t idx = lane; idx < ed * d; idx += 64) {
    const uint32_t l = div_small(idx, rd), pos = idx - l * d;
    uint8_t v;
    if (pos >= npd) {
      v = s.Ba[l * w + ed + (pos - npd)];
    } else {
      v = 0;
      const uint32_t pc = s.Pl[pos];
      uint32_t acc = 0;
#pragma unroll 4
      for (uint32_t i = 0; i < ed; ++i) acc ^= lmul(lg, ex, s.Ba[l * w + ed + i], M[s.Jl[i] * d + pc]);
      v = static_cast<uint8_t>(acc);
    }
    s.DE[l * 64 + pos] = v;
  }
  wsync();
  // header + rows + coefficients
  const uint32_t dpad = a.dpad, epad = a.epad;
  if (lane == 0) *reinterpret_cast<uint32_t*>(desc) = (e & 0xffu) | (ed << 8);
  for (uint32_t i = lane; i < dpad; i += 64) desc[4 + i] = i < d ? s.surv[i] : 0;
  for (uint32_t i = lane; i < epad; i += 64) desc[4 + dpad + i] = i < e ? s.outr[i] : 0;
  DescPtr coef = desc + 4 + dpad + epad;
  for (uint32_t idx = lane; idx < e * dpad; idx += 64) {
    const uint32_t i = div_small(idx, rdp), pos = idx - i * dpad;
    uint8_t v = 0;
    if (pos < d) {
      if (i < ed) {
        v = s.DE[i * 64 + pos];
      } else {
        const uint32_t r = s.outr[i];
        if (pos < npd) v = M[r * d + s.Pl[pos]];
        uint32_t acc = v;
#pragma unroll 4
        for (uint32_t l = 0; l < ed; ++l) acc ^= lmul(lg, ex, M[r * d + s.El[l]], s.DE[l * 64 + pos]);
        v = static_cast<uint8_t>(acc);
      }
    }
    coef[idx] = v;
  }
}

// kPrepWaves groups per block, one per wave: the tables and M are staged
// once per block, and 8192 jumbo groups fit the chip in about one round
// (22 KiB of LDS per block).
constexpr uint32_t kPrepWaves = 4;

template <int EDM, int NMD, int WPE = 1>
__global__ __launch_bounds__(64 * kPrepWaves) __attribute__((amdgpu_waves_per_eu(WPE))) void k_prepare(Prep a,
                                                                                                       uint32_t groups) {
  __shared__ PrepSharedT<NMD> sh;
  __shared__ PrepWaveT<EDM> sw[kPrepWaves];
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63u;
  prep_stage(a, sh, threadIdx.x, 64 * kPrepWaves);
  __syncthreads();
  const uint32_t gl = blockIdx.x * kPrepWaves + w;
  if (gl >= groups) return;
  const uint64_t g = a.g0 + gl;
  prep_wave(a, g, a.desc + (g - a.g_desc0) * a.desc_stride, sh, sw[w], lane);
}

// ------------------------------------------------------------- launchers
LaunchTimer*& current_timer() {
  static thread_local LaunchTimer* t = nullptr;
  return t;
}

static inline uint32_t blocks_for(uint64_t items, uint32_t bs) {
  return static_cast<uint32_t>((items + bs - 1) / bs);
}

// Launch policy (tuned with tools/kvariants.hip on MI355X, DESIGN_HISTORY.md §3.4).
// Store policy is chosen for the cold-HBM regime -- a batch whose lines are
// not in the 256-MB Infinity Cache, as every fresh batch of packets is
// (`kvariants 65536 21 cold`, each sample after a cache-evicting sweep):
// nontemporal stores there take the (10,3) encode from 217.9 to 197.3 us and
// the reconstruct from 228.4 to 201.0 us.  Re-running
// ONE batch back to back instead (a warm loop) favours plain stores by 3-5%,
// because the Infinity Cache then absorbs the rewritten parity lines.
constexpr int kEncNT = 3;    // nontemporal loads and stores
#ifndef UGO_ENC_LDS_ROWS  // A/B builds only (tools/bench_ab.sh with UGO_FEC_LIB)
#define UGO_ENC_LDS_ROWS 8
#endif
#ifndef UGO_ENC_STAGE_ROWS
#define UGO_ENC_STAGE_ROWS 13
#endif
constexpr int kEncLdsRows = UGO_ENC_LDS_ROWS;  // (10,3): rows 0-7 by LDS-DMA nt, 8-9 to registers
constexpr int kEncStageRows = UGO_ENC_STAGE_ROWS;  // (10,3): 52-KiB stage, 3 blocks per CU (see k_encode_g)
constexpr int kEncJumboNT = 3;  // (32,8): NT loads and stores (578 vs 615 us, tools/jvariants.hip)
// (32,8): the network in Four-Russians form with the dwords in sequence
// (k_encode_frs), rows 0-15 by LDS-DMA nt and read from LDS one dword at a
// time (blocks of 3: 133 VGPRs), 2 blocks per CU (64-KiB stage): 519.9 / 524.6 us against
// 548.9 / 567.2 us for the Horner network k_encode_g with 8 staged rows on two
// boxes, byte-identical parity (profiles/r2/jvariants_frs*.jsonl).  The
// Horner network's own pick was 8 staged rows (565 vs 584 us for 16 in 9 of
// 12 interleaved runs, profiles/r2/jvariants_lds_rows_r2.txt).
constexpr int kEncJumboLdsRows = 16;
// Four-Russians blocks of 2 inputs (a, b, a^b): more XORs than blocks of 3
// but 108 instead of 133 VGPRs, 519.4 / 517.9 us against 527.8 / 524.7 (blocks
// of 4: 532.3) in two interleaved runs (profiles/r2/jvariants_fr_blocks*.jsonl)
constexpr int kEncJumboFrBlock = 2;
constexpr int kApplyNT = 3;  // nontemporal loads and stores
constexpr int kApplyPNT = 3; // k_apply_p: nontemporal loads and stores (cold: 201.0 vs 228.4 us)
constexpr int kApplyQNT = 3; // k_apply_q (jumbo): NT loads and stores (548 vs 572 us)

int apply_dmax(int d) {
  if (d <= 4) return 4;
  if (d <= 8) return 8;
  if (d <= 10) return 10;
  if (d <= 12) return 12;
  if (d <= 16) return 16;
  if (d <= 24) return 24;
  if (d <= 32) return 32;
  return 0;
}

bool has_const_encode(int d, int p) { return (d == 10 && p == 3) || (d == 32 && p == 8); }

hipError_t launch_encode_const(int d, int p, const Batch& a, hipStream_t s) {
  const dim3 grid(blocks_for(a.items, 256)), block(256);
  if (d == 10 && p == 3)
    launch(kKEncode, k_encode_g<10, 3, kEncNT & 2, kEncLdsRows, 256, kEncStageRows>, grid, block, 0, s, a);
  else if (d == 32 && p == 8)
    launch(kKEncode, k_encode_frs<32, 8, kEncJumboNT & 2, kEncJumboLdsRows, 256, kEncJumboLdsRows, 2, kEncJumboFrBlock>,
           grid, block, 0, s, a);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

// Streaming kernels for wide codes (chunks >= 64, e <= 8 outputs): registers
// do not grow with d, so any d (up to 255) runs here.  False if not eligible.
// MODE 0 applies the encode descriptor: timed as an encode
template <int MODE>
constexpr KernelId apply_kid() { return MODE == 0 ? kKEncode : kKReconstruct; }

template <int MODE>
static bool launch_apply_stream(const Batch& a, hipStream_t s) {
  if (a.chunks < 64 || a.epad > 8) return false;
  const dim3 block(256);
  const uint32_t cpad = (a.chunks + 63u) & ~63u;
  if (MODE != 0 && (cpad - a.chunks) * 16u <= cpad) {  // groups wave-aligned at <= 1/16 idle lanes
    Batch b = a;
    b.items = (a.items / a.chunks) * cpad;
    const dim3 ga((blocks_for(b.items, 256) + 7u) & ~7u);  // OPT & 32: a multiple of 8
    // k_apply_qb: k_apply_qa with its per-product overhead cut (uniform
    // descriptor in SGPRs, saddr loads, unrolled ring): jumbo reconstruct
    // 524.0 vs 535.5 us (profiles/r3/qaprobe_r3e.jsonl); and each XCD on one
    // contiguous eighth of the groups, so a group's blocks share one L2 for
    // its descriptor: 482-523 vs 505-533 us over 8 allocations
    // (profiles/r3/qaprobe_xcd.jsonl)
    if (a.epad == 4)
      launch(apply_kid<MODE>(), k_apply_qb<4, MODE, kApplyQNT, 39>, ga, block, 0, s, b);
    else
      launch(apply_kid<MODE>(), k_apply_qb<8, MODE, kApplyQNT, 39>, ga, block, 0, s, b);
    return true;
  }
  const dim3 grid(blocks_for(a.items, 256));
  if (a.epad == 4)
    launch(apply_kid<MODE>(), k_apply_q<4, MODE, kApplyQNT, 1>, grid, block, 0, s, a);
  else
    launch(apply_kid<MODE>(), k_apply_q<8, MODE, kApplyQNT, 1>, grid, block, 0, s, a);
  return true;
}

// k_apply_w needs a wave to span <= 2 groups (>= 64 chunks per row) and all
// output rows in one descriptor dword (p <= 4); k_apply covers the rest.
template <int DMAX, int MODE>
static void launch_apply_dm(const Batch& a, hipStream_t s) {
  const dim3 grid(blocks_for(a.items, 256)), block(256);
  if constexpr (DMAX <= 16) {
    if (a.chunks >= 64 && a.epad == 4) {
      launch(apply_kid<MODE>(), k_apply_p<DMAX, MODE, kApplyPNT, 1>, grid, block, 0, s, a);
      return;
    }
  }
  if (launch_apply_stream<MODE>(a, s)) return;  // wide codes: streaming inputs
  if (a.chunks >= 64 && a.epad == 4) {
    Batch b = a;
    b.pass = (a.items + 63u) / 64u * 64u;
    launch(apply_kid<MODE>(), k_apply_w<DMAX, MODE, kApplyNT, 1>, grid, block, 0, s, b);
  }
  else
    launch(apply_kid<MODE>(), k_apply<DMAX, MODE, kApplyNT>, grid, block, 0, s, a);
}

template <int MODE>
static hipError_t launch_apply_mode(int dmax, const Batch& a, hipStream_t s) {
  switch (dmax) {
    case 0:  // d > 32: the streaming kernels, any row length and output count
      if (!launch_apply_stream<MODE>(a, s)) {
        // rows < 64 chunks or > 8 outputs: wave-aligned groups (idle lanes past
        // a short row), outputs folded 8 at a time
        Batch b = a;
        const uint32_t cpad = (a.chunks + 63u) & ~63u;
        b.items = (a.items / a.chunks) * cpad;
        launch(apply_kid<MODE>(), k_apply_qa<8, MODE, kApplyQNT, 2, 1, true>, dim3(blocks_for(b.items, 256)),
               dim3(256), 0, s, b);
      }
      break;
    case 4: launch_apply_dm<4, MODE>(a, s); break;
    case 8: launch_apply_dm<8, MODE>(a, s); break;
    case 10: launch_apply_dm<10, MODE>(a, s); break;
    case 12: launch_apply_dm<12, MODE>(a, s); break;
    case 16: launch_apply_dm<16, MODE>(a, s); break;
    case 24: launch_apply_dm<24, MODE>(a, s); break;
    case 32: launch_apply_dm<32, MODE>(a, s); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_apply(int mode, int dmax, const Batch& a, hipStream_t s) {
  switch (mode) {
    case 0: return launch_apply_mode<0>(dmax, a, s);
    case 1: return launch_apply_mode<1>(dmax, a, s);
    case 2: return launch_apply_mode<2>(dmax, a, s);
    default: return hipErrorInvalidValue;
  }
}

// ------------------------------------------------------------- list form
// Lossy-group list in two launches, ascending group order, no global atomics:
// block b of k_lossy_count counts the groups of its kLossyPerBlock that have an
// erased row to rebuild, and the rows they rebuild; block b of k_lossy_write
// sums both counts over the blocks < b (its output offsets), scans its own
// groups in order and writes their indices (and row offsets); the last block
// also writes the totals.
__device__ __forceinline__ uint32_t lossy_rows(uint64_t m, uint64_t nmask, uint64_t dmask, uint32_t d,
                                               bool& lossy) {
  const uint64_t lost = ~m & nmask & dmask;
  lossy = lost != 0;
  return static_cast<uint32_t>(__popcll(m & nmask)) >= d ? static_cast<uint32_t>(__popcll(lost)) : 0u;
}

__global__ __launch_bounds__(1024) void k_lossy_count(const uint64_t* present, uint64_t groups, uint64_t nmask,
                                                      uint64_t dmask, uint32_t d, uint32_t* work) {
  __shared__ uint32_t tot[2];
  if (threadIdx.x < 2) tot[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t g0 = uint64_t(blockIdx.x) * kLossyPerBlock;
  uint32_t c = 0, r = 0;
  for (uint32_t k = threadIdx.x; k < kLossyPerBlock; k += 1024u) {
    const uint64_t g = g0 + k;
    if (g >= groups) break;
    bool l;
    const uint32_t rows = lossy_rows(present[g], nmask, dmask, d, l);
    c += l;
    r += rows;
  }
  c = __reduce_add_sync(~0ull, c);
  r = __reduce_add_sync(~0ull, r);
  if ((threadIdx.x & 63u) == 0) {
    if (c) atomicAdd(&tot[0], c);
    if (r) atomicAdd(&tot[1], r);
  }
  __syncthreads();
  if (threadIdx.x < 2) work[2 * blockIdx.x + threadIdx.x] = tot[threadIdx.x];
}

// inclusive scan over a 64-lane wave
__device__ __forceinline__ uint32_t wave_inclusive(uint32_t v, uint32_t lane) {
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t u = __shfl_up(v, off, 64);
    if (static_cast<int>(lane) >= off) v += u;
  }
  return v;
}

// Thread t scans groups g0 + 4t .. g0 + 4t + 3 (kLossyPerBlock / 1024 = 4 per
// thread, in order); block-wide exclusive scans of the per-thread counts place
// them.
__global__ __launch_bounds__(1024) void k_lossy_write(const uint64_t* present, uint64_t groups, uint64_t nmask,
                                                      uint64_t dmask, uint32_t d, const uint32_t* work,
                                                      uint32_t* list, uint32_t* count, uint32_t* rowoff,
                                                      uint32_t* rows_total) {
  constexpr uint32_t kPer = kLossyPerBlock / 1024u;
  __shared__ uint32_t wsum[2][16];
  __shared__ uint32_t base[2];
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  // this block's offsets: the counts of all earlier blocks
  uint32_t before = 0, rbefore = 0;
  for (uint32_t b = t; b < blockIdx.x; b += 1024u) {
    before += work[2 * b];
    rbefore += work[2 * b + 1];
  }
  before = __reduce_add_sync(~0ull, before);
  rbefore = __reduce_add_sync(~0ull, rbefore);
  if (t < 2) base[t] = 0;
  __syncthreads();
  if (lane == 0) {
    if (before) atomicAdd(&base[0], before);
    if (rbefore) atomicAdd(&base[1], rbefore);
  }
  const uint64_t g0 = uint64_t(blockIdx.x) * kLossyPerBlock + uint64_t(t) * kPer;
  uint32_t bits = 0, c = 0, r = 0, rk[kPer];
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    const uint64_t g = g0 + k;
    bool l = false;
    rk[k] = g < groups ? lossy_rows(present[g], nmask, dmask, d, l) : 0u;
    bits |= static_cast<uint32_t>(l) << k;
    c += l;
    r += rk[k];
  }
  const uint32_t inc = wave_inclusive(c, lane), rinc = wave_inclusive(r, lane);
  if (lane == 63u) {
    wsum[0][wv] = inc;
    wsum[1][wv] = rinc;
  }
  __syncthreads();
  uint32_t wbefore = 0, wrbefore = 0;
  for (uint32_t w = 0; w < wv; ++w) {
    wbefore += wsum[0][w];
    wrbefore += wsum[1][w];
  }
  uint32_t pos = base[0] + wbefore + inc - c, rpos = base[1] + wrbefore + rinc - r;
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k)
    if ((bits >> k) & 1u) {
      list[pos] = static_cast<uint32_t>(g0 + k);
      if (rowoff) rowoff[pos] = rpos;
      ++pos;
      rpos += rk[k];
    }
  if (blockIdx.x == gridDim.x - 1u && t == 1023u) {  // the last thread's ends = the totals
    *count = pos;
    if (rows_total) *rows_total = rpos;
  }
}

// The same list in ONE launch (round 6): block b counts its
// tile, publishes (count, rows) tagged with the call's epoch in one 64-bit word
// (epoch << 32 | rows << 13 | count: a tile holds at most 4096 groups, 13 bits,
// and 4096 * 32 rows, 18 bits), then waits until every block before it has
// published and sums their words in parallel (block b reads b words over its
// 1024 threads) -- no chained look-back, so no block waits on another's wait.
// Forward progress: a block publishes before it waits, and the lowest block
// that has not published is always dispatched (workgroups go out in index
// order, so the blocks holding its XCD's slots are lower ones, which have
// published and only wait on published blocks).  The words live in
// context-owned memory, one buffer per stream (calls on one stream are ordered;
// the epoch grows per call, so a word from an earlier call never matches).
__global__ __launch_bounds__(1024) void k_lossy_list1(const uint64_t* present, uint64_t groups, uint64_t nmask,
                                                      uint64_t dmask, uint32_t d, uint64_t* words, uint32_t epoch,
                                                      uint32_t* list, uint32_t* count, uint32_t* rowoff,
                                                      uint32_t* rows_total) {
  constexpr uint32_t kPer = kLossyPerBlock / 1024u;
  __shared__ uint32_t wsum[2][16];
  __shared__ uint32_t base[2];
  const uint32_t t = threadIdx.x, lane = t & 63u, wv = t >> 6;
  const uint64_t g0 = uint64_t(blockIdx.x) * kLossyPerBlock + uint64_t(t) * kPer;
  uint32_t bits = 0, c = 0, r = 0, rk[kPer];
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    const uint64_t g = g0 + k;
    bool l = false;
    rk[k] = g < groups ? lossy_rows(present[g], nmask, dmask, d, l) : 0u;
    bits |= static_cast<uint32_t>(l) << k;
    c += l;
    r += rk[k];
  }
  const uint32_t inc = wave_inclusive(c, lane), rinc = wave_inclusive(r, lane);
  if (lane == 63u) {
    wsum[0][wv] = inc;
    wsum[1][wv] = rinc;
  }
  if (t < 2) base[t] = 0;
  __syncthreads();
  if (t == 0) {  // this tile's totals, published at once
    uint32_t tc = 0, tr = 0;
    for (uint32_t w = 0; w < 16u; ++w) {
      tc += wsum[0][w];
      tr += wsum[1][w];
    }
    const uint64_t word = (uint64_t(epoch) << 32) | (uint64_t(tr) << 13) | tc;
    __hip_atomic_store(&words[blockIdx.x], word, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
  // every earlier tile's totals: thread t waits for tiles t, t + 1024, ... below this one
  uint32_t before = 0, rbefore = 0;
  for (uint32_t b = t; b < blockIdx.x; b += 1024u) {
    uint64_t w;
    uint32_t spins = 0;
    do {
      w = __hip_atomic_load(&words[b], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      if (static_cast<uint32_t>(w >> 32) != epoch) {
        __builtin_amdgcn_s_sleep(1);
        // a word that never arrives (seconds) is a broken invariant: fault loudly instead of hanging
        if (++spins == (1u << 26)) __builtin_trap();
      }
    } while (static_cast<uint32_t>(w >> 32) != epoch);
    before += static_cast<uint32_t>(w) & 0x1fffu;
    rbefore += static_cast<uint32_t>(w) >> 13;
  }
  before = __reduce_add_sync(~0ull, before);
  rbefore = __reduce_add_sync(~0ull, rbefore);
  if (lane == 0) {
    if (before) atomicAdd(&base[0], before);
    if (rbefore) atomicAdd(&base[1], rbefore);
  }
  __syncthreads();
  uint32_t wbefore = 0, wrbefore = 0;
  for (uint32_t w = 0; w < wv; ++w) {
    wbefore += wsum[0][w];
    wrbefore += wsum[1][w];
  }
  uint32_t pos = base[0] + wbefore + inc - c, rpos = base[1] + wrbefore + rinc - r;
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k)
    if ((bits >> k) & 1u) {
      list[pos] = static_cast<uint32_t>(g0 + k);
      if (rowoff) rowoff[pos] = rpos;
      ++pos;
      rpos += rk[k];
    }
  if (blockIdx.x == gridDim.x - 1u && t == 1023u) {  // the last thread's ends = the totals
    *count = pos;
    if (rows_total) *rows_total = rpos;
  }
}

hipError_t launch_lossy_list1(const uint64_t* present, uint64_t groups, uint64_t nmask, uint64_t dmask, uint32_t d,
                              uint32_t* list, uint32_t* count, uint32_t* rowoff, uint32_t* rows, uint64_t* words,
                              uint32_t epoch, hipStream_t s) {
  const uint64_t blocks = (groups + kLossyPerBlock - 1) / kLossyPerBlock;
  if (blocks == 0 || blocks > 0xffffffffull) return hipErrorInvalidValue;
  launch(kKReconstruct, k_lossy_list1, dim3(static_cast<uint32_t>(blocks)), dim3(1024), 0, s, present, groups, nmask,
         dmask, d, words, epoch, list, count, rowoff, rows);
  return hipGetLastError();
}

hipError_t launch_lossy_list(const uint64_t* present, uint64_t groups, uint64_t nmask, uint64_t dmask, uint32_t d,
                             uint32_t* list, uint32_t* count, uint32_t* rowoff, uint32_t* rows, uint32_t* work,
                             hipStream_t s) {
  const uint64_t blocks = (groups + kLossyPerBlock - 1) / kLossyPerBlock;
  if (blocks == 0 || blocks > 0xffffffffull) return hipErrorInvalidValue;
  launch(kKReconstruct, k_lossy_count, dim3(static_cast<uint32_t>(blocks)), dim3(1024), 0, s, present, groups, nmask,
         dmask, d, work);
  launch(kKReconstruct, k_lossy_write, dim3(static_cast<uint32_t>(blocks)), dim3(1024), 0, s, present, groups, nmask,
         dmask, d, static_cast<const uint32_t*>(work), list, count, rowoff, rows);
  return hipGetLastError();
}

template <int DMAX>
static void launch_apply_list_dm(const Batch& a, hipStream_t s) {
  const dim3 grid(blocks_for(a.items, 256)), block(256);
  if (a.chunks >= 64 && a.epad == 4)
    launch(kKReconstruct, k_apply_p<DMAX, 1, kApplyPNT, 1, 1, 4, true, 0, 0, true>, grid, block, 0, s, a);
  else
    launch(kKReconstruct, k_apply<DMAX, 1, kApplyNT, true>, grid, block, 0, s, a);
}

hipError_t launch_apply_list(int dmax, const Batch& a, hipStream_t s) {
  switch (dmax) {
    case 4: launch_apply_list_dm<4>(a, s); break;
    case 8: launch_apply_list_dm<8>(a, s); break;
    case 10: launch_apply_list_dm<10>(a, s); break;
    case 12: launch_apply_list_dm<12>(a, s); break;
    case 16: launch_apply_list_dm<16>(a, s); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <int MODE>
static hipError_t launch_apply_dense_mode(int dmax, const Batch& a, hipStream_t s) {
  const uint32_t waves = (a.items + 62u) / 63u;
  const dim3 grid((waves + 3u) / 4u), block(256);
  switch (dmax) {
    case 4: launch(kKReconstruct, k_apply_pd<4, MODE, kApplyPNT>, grid, block, 0, s, a); break;
    case 8: launch(kKReconstruct, k_apply_pd<8, MODE, kApplyPNT>, grid, block, 0, s, a); break;
    case 10: launch(kKReconstruct, k_apply_pd<10, MODE, kApplyPNT>, grid, block, 0, s, a); break;
    case 12: launch(kKReconstruct, k_apply_pd<12, MODE, kApplyPNT>, grid, block, 0, s, a); break;
    case 16: launch(kKReconstruct, k_apply_pd<16, MODE, kApplyPNT>, grid, block, 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_apply_dense(int mode, int dmax, const Batch& a, hipStream_t s) {
  if (a.S < kDenseMinS || a.epad != 4) return hipErrorInvalidValue;
  switch (mode) {
    case 1: return launch_apply_dense_mode<1>(dmax, a, s);
    case 2: return launch_apply_dense_mode<2>(dmax, a, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_service(int dmax, const SvcArgs& sa, hipStream_t s) {
  if (sa.a.epad != 4) return hipErrorInvalidValue;
  const dim3 grid(1), block(kSvcThreads);
  switch (dmax) {  // never timed: it stays resident across calls
    case 4: hipLaunchKernelGGL(k_service<4>, grid, block, 0, s, sa); break;
    case 8: hipLaunchKernelGGL(k_service<8>, grid, block, 0, s, sa); break;
    case 10: hipLaunchKernelGGL(k_service<10>, grid, block, 0, s, sa); break;
    case 12: hipLaunchKernelGGL(k_service<12>, grid, block, 0, s, sa); break;
    case 16: hipLaunchKernelGGL(k_service<16>, grid, block, 0, s, sa); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_apply_bytes(int mode, const Batch& a, hipStream_t s) {
  const dim3 grid(blocks_for(a.items, 256)), block(256);
  switch (mode) {
    case 0: launch(kKBytes, k_apply_bytes<0>, grid, block, 0, s, a); break;
    case 1: launch(kKBytes, k_apply_bytes<1>, grid, block, 0, s, a); break;
    case 2: launch(kKBytes, k_apply_bytes<2>, grid, block, 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_apply_rows(int mode, const Batch& a, hipStream_t s) {
  Batch b = a;  // wave-aligned groups
  b.items = (a.items / a.chunks) * ((a.chunks + 63u) & ~63u);
  const dim3 grid(blocks_for(b.items, 256)), block(256);
  switch (mode) {
    case 1: launch(kKReconstruct, k_apply_rows<1>, grid, block, 0, s, b); break;
    case 2: launch(kKReconstruct, k_apply_rows<2>, grid, block, 0, s, b); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_prepare(const Prep& a, uint32_t groups, hipStream_t s) {
  const dim3 grid((groups + kPrepWaves - 1) / kPrepWaves), block(64 * kPrepWaves);
  if (std::min(a.d, a.n - a.d) <= static_cast<uint32_t>(kPrepSmallEdm) && a.n * a.d <= static_cast<uint32_t>(kPrepSmallNmd))
    launch(kKPrepare, k_prepare<kPrepSmallEdm, kPrepSmallNmd, kPrepSmallWpe>, grid, block, 0, s, a, groups);
  else
    launch(kKPrepare, k_prepare<32, 64 * 64>, grid, block, 0, s, a, groups);
  return hipGetLastError();
}

}  // namespace kern
}  // namespace ugo
