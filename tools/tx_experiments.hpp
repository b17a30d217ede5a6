// tx_experiments.hpp -- k_tx_g, the one-block-per-group TX assembly measured
// in round 4 against production's k_tx_c and not shipped (tools/txgroup.hip;
// profiles/r4/txgroup_*.jsonl: 495-500 us against 432-438 us).  Included after
// ugo_amd/csrc/tx_kernels.hip, whose helpers it uses.  Not product code.
#pragma once

namespace ugo {
namespace kern {

template <int D, int P, int NT, int... I>
__device__ __forceinline__ void tx_g_parity(uint8_t* p0, uint64_t slot, const V4* x, const V4& padc, uint32_t m,
                                            uint32_t seq, uint32_t keep, std::integer_sequence<int, I...>) {
  (
      [&] {
        V4 y = cparity<D, P, I>(x);
        if (m == 0) put_header(y, seq + I, kTypeFEC);
        xor4(y, padc);
        store16<NT>(p0 + uint64_t(I) * slot, keep_bytes(y, keep), 16u);
      }(),
      ...);
}

// One block per group (k_tx_g): the group's d data packets are one contiguous
// run of the input ring and its d + p wire packets one contiguous run of the
// output, so the block streams both in order -- each pass of 256 threads
// reads 4 KiB of data packets and writes the same 4 KiB of wire packets
// (header, pad), keeping the parity inputs (header bytes and bytes past each
// length zeroed) in LDS; after one barrier, the threads of chunks [0, maxsz)
// fold the d LDS rows through the compile-time network into the p parity
// packets, written after the data packets.  Per group d x chunks x 16 B of
// LDS (14.9 KiB for (10,3) x 1476).  Semantics exactly k_tx_c's.
constexpr uint32_t kTxGroupLds = 48 * 1024;

template <int D, int P, int NT = kTxNT>
__global__ __launch_bounds__(256) void k_tx_g(TxArgs a) {
  extern __shared__ u32x4 xs[];  // [D][chunks]
  const uint64_t g = a.g0 + blockIdx.x;
  const uint32_t t = threadIdx.x;
  const uint32_t nch = a.chunks, n = D + P;
  uint32_t Ls[D];
  bool bad = false;
  uint32_t maxsz = 0;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    Ls[k] = a.lens[g * D + k];  // uniform: scalar loads
    bad |= Ls[k] < 6u || Ls[k] > a.max_len;
    maxsz = max(maxsz, Ls[k]);
  }
  if (bad) {  // a length outside [6, max_len]: nothing goes out for this group
    if (t == 0 && a.status) a.status[g] = kBadLength;
    if (t < n) a.wire_lens[g * n + t] = 0;
    return;
  }
  const uint32_t seq0 = static_cast<uint32_t>((uint64_t(a.first_seq) + g * n) % a.paws);
  const uint8_t* src = a.pkts + g * D * a.slot_in;
  uint8_t* dst = a.wire + g * n * a.slot_out;
  constexpr int kPass = (D * 96 + 255) / 256;  // passes over d x chunks (chunks <= 96 for unrolled loads)
  // data packets: all loads of the thread first, then the stores and LDS rows
  if (nch <= 96) {
    V4 x[kPass];
#pragma unroll
    for (int q = 0; q < kPass; ++q) {
      const uint32_t idx = t + 256u * q, k = idx / nch, m = idx - k * nch, o = 16u * m;
      x[q] = V4{{0u, 0u, 0u, 0u}};
      if (k < static_cast<uint32_t>(D) && o < Ls[k]) x[q] = load16<1>(src + uint64_t(k) * a.slot_in + o);
    }
#pragma unroll
    for (int q = 0; q < kPass; ++q) {
      const uint32_t idx = t + 256u * q, k = idx / nch, m = idx - k * nch, o = 16u * m;
      if (k >= static_cast<uint32_t>(D)) continue;
      const uint32_t Lk = Ls[k];
      V4 v = keep_bytes(x[q], Lk - min(Lk, o));
      if (o < Lk) {
        V4 w = v;
        if (m == 0) put_header(w, seq0 + k, kTypeData);
        if (a.pad) xor4(w, load16<0>(a.pad + o));
        store16<NT>(dst + uint64_t(k) * a.slot_out + o, keep_bytes(w, Lk - o), 16u);
      }
      if (m == 0) {
        v.v[0] = 0u;
        v.v[1] &= 0xffff0000u;
      }
      xs[k * nch + m] = u32x4{v.v[0], v.v[1], v.v[2], v.v[3]};
    }
  } else {
    for (uint32_t idx = t; idx < D * nch; idx += 256u) {
      const uint32_t k = idx / nch, m = idx - k * nch, o = 16u * m;
      const uint32_t Lk = Ls[k];
      V4 v = V4{{0u, 0u, 0u, 0u}};
      if (o < Lk) v = keep_bytes(load16<1>(src + uint64_t(k) * a.slot_in + o), Lk - o);
      if (o < Lk) {
        V4 w = v;
        if (m == 0) put_header(w, seq0 + k, kTypeData);
        if (a.pad) xor4(w, load16<0>(a.pad + o));
        store16<NT>(dst + uint64_t(k) * a.slot_out + o, keep_bytes(w, Lk - o), 16u);
      }
      if (m == 0) {
        v.v[0] = 0u;
        v.v[1] &= 0xffff0000u;
      }
      xs[k * nch + m] = u32x4{v.v[0], v.v[1], v.v[2], v.v[3]};
    }
  }
  if (t < static_cast<uint32_t>(D)) a.wire_lens[g * n + t] = static_cast<uint16_t>(Ls[t]);
  if (maxsz <= kFecHeader) {  // header-only group: no parity (tx_no_window)
    if (t == 0 && a.status) a.status[g] = kNoData;
    if (t < static_cast<uint32_t>(P)) a.wire_lens[g * n + D + t] = 0;
    return;
  }
  __syncthreads();
  for (uint32_t m = t; m < nch; m += 256u) {
    const uint32_t o = 16u * m;
    if (o >= maxsz) break;
    V4 x[D];
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const u32x4 v = xs[k * nch + m];
      x[k] = V4{{v.x, v.y, v.z, v.w}};
    }
    const V4 padc = a.pad ? load16<0>(a.pad + o) : V4{{0u, 0u, 0u, 0u}};
    tx_g_parity<D, P, NT>(dst + uint64_t(D) * a.slot_out + o, a.slot_out, x, padc, m, seq0 + D, maxsz - o,
                          std::make_integer_sequence<int, P>{});
  }
  if (t < static_cast<uint32_t>(P)) a.wire_lens[g * n + D + t] = static_cast<uint16_t>(maxsz);
  if (t == 0 && a.status) a.status[g] = 0;
}

}  // namespace kern
}  // namespace ugo
