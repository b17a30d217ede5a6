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
// One wave per packet: every lane owns 16-byte chunks of the payload.  The
// packet sits at a 16-aligned slot, so its payload (offset 6) is misaligned;
// each lane loads the two aligned chunks covering its 16 output bytes, XORs
// the keystream chunks, and realigns with v_alignbyte.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "rx_kernels.hpp"

namespace ugo {
namespace kern {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 ld16(const uint8_t* p) { return *reinterpret_cast<const u32x4*>(p); }

__global__ __launch_bounds__(256) void k_rx_scatter(RxArgs a) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = (blockIdx.x * 256ull + threadIdx.x) >> 6;
  const uint64_t nwaves = (gridDim.x * 256ull) >> 6;
  const uint32_t nq = (a.S + 15u) / 16u;  // output chunks per row
  for (uint64_t i = wave; i < a.npk; i += nwaves) {
    const uint8_t* pk = a.wire + i * a.slot;
    const uint32_t len = a.lens[i];
    if (len < 6u) {
      if (lane == 0 && a.stats) atomicAdd(&a.stats[3], 1u);
      continue;
    }
    u32x4 h = ld16(pk);
    if (a.pad) h ^= ld16(a.pad);
    const uint32_t seqid = h.x;
    const uint32_t flag = h.y & 0xffffu;
    if (flag != 0xf1u && flag != 0xf2u) {  // ugo/conn.go:395
      if (lane == 0 && a.stats) atomicAdd(&a.stats[1], 1u);
      continue;
    }
    const uint32_t row = seqid % a.n;
    const uint64_t grp = seqid / a.n;
    if (grp < a.first_group || grp >= a.first_group + a.groups) {
      if (lane == 0 && a.stats) atomicAdd(&a.stats[2], 1u);
      continue;
    }
    const uint64_t gs = grp - a.first_group;
    uint8_t* dst = a.shards + row * a.rstride + gs * a.gstride;
    const uint32_t L = min(len - 6u, a.S);  // copy(buf, data[6:]) bounded by the row
    for (uint32_t q = lane; q < nq; q += 64u) {
      const uint32_t o = 16u * q;  // payload byte offset of this chunk
      u32x4 A = {0u, 0u, 0u, 0u}, B = {0u, 0u, 0u, 0u};
      if (o < L) {
        A = ld16(pk + o);
        if (a.pad) A ^= ld16(a.pad + o);
        if (o + 16u < a.slot) {
          B = ld16(pk + o + 16u);
          if (a.pad) B ^= ld16(a.pad + o + 16u);
        }
      }
      // payload bytes [o, o+16) = packet bytes [o+6, o+22)
      uint32_t w[4];
      w[0] = __builtin_amdgcn_alignbyte(A.z, A.y, 2);
      w[1] = __builtin_amdgcn_alignbyte(A.w, A.z, 2);
      w[2] = __builtin_amdgcn_alignbyte(B.x, A.w, 2);
      w[3] = __builtin_amdgcn_alignbyte(B.y, B.x, 2);
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
    if (lane == 0) {
      atomicOr(reinterpret_cast<unsigned long long*>(&a.present[gs]), 1ull << row);
      if (a.stats) atomicAdd(&a.stats[0], 1u);
    }
  }
}

hipError_t launch_rx_scatter(const RxArgs& a, hipStream_t s) {
  const uint64_t waves = a.npk;
  uint32_t blocks = static_cast<uint32_t>((waves + 3) / 4);
  if (blocks > 8192u) blocks = 8192u;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rx_scatter, dim3(blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace kern
}  // namespace ugo
