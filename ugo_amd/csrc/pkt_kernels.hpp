// pkt_kernels.hpp -- internal interface of the packet wire-codec decoder.
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstdint>

#include "../../include/ugo_pkt.h"

namespace ugo {
namespace kern {

struct PktArgs {
  const uint8_t* pkts;     // packet i at pkts + i*slot (16-B aligned)
  const uint16_t* lens;
  const uint8_t* pad;      // nullable keystream, >= slot bytes
  ugo_pkt_info* info;
  uint64_t* ranges;        // [npk][max_ranges][2]
  ugo_pkt_segment* segs;   // [npk][max_segments]
  uint64_t npk;
  uint64_t slot;
  uint32_t max_ranges;
  uint32_t max_segments;
  uint32_t framed;
};

hipError_t launch_packet_decode(const PktArgs& a, hipStream_t s);

}  // namespace kern
}  // namespace ugo
