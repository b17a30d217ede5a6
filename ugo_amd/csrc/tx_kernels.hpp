// tx_kernels.hpp -- internal interface of the TX group-assembly kernel.
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstdint>

namespace ugo {
namespace kern {

struct TxArgs {
  const uint8_t* pkts;   // data packet k of group g at pkts + (g*d + k)*slot_in (16-B aligned)
  const uint16_t* lens;  // [G*d] packet lengths, 6-B header space included
  const uint8_t* pad;    // keystream XORed over every wire packet from byte 0, or null
  const uint8_t* desc;   // MODE 0 encode descriptor (geometries without a fixed network)
  uint8_t* wire;         // wire packet r of group g at wire + (g*n + r)*slot_out
  uint16_t* wire_lens;   // [G*n]
  int8_t* status;        // [G], nullable
  uint64_t groups;
  uint64_t g0;           // first group of this launch (seqids count from group 0)
  uint64_t slot_in;
  uint64_t slot_out;
  uint32_t first_seq;    // seqid of group 0's first data packet (multiple of n, < paws)
  uint32_t paws;         // (0xffffffff / n - 1) * n
  uint32_t max_len;      // longest accepted data packet
  uint32_t chunks;       // ceil(max_len / 16)
  uint32_t d, p, dpad, epad;
};

// dmax: 0 selects the compile-time networks (10,3) / (32,8); otherwise the
// descriptor kernel instantiated for d <= dmax.
hipError_t launch_tx_assemble(int dmax, const TxArgs& a, hipStream_t s);

}  // namespace kern
}  // namespace ugo
