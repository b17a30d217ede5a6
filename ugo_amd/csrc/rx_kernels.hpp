// rx_kernels.hpp -- internal interface of the RX group-assembly kernel.
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstdint>

namespace ugo {
namespace kern {

struct RxArgs {
  const uint8_t* wire;     // packet i at wire + i*slot (device, 16-B aligned slots)
  const uint16_t* lens;    // packet lengths (device)
  const uint8_t* pad;      // keystream XORed over each packet from byte 0, >= slot bytes, or null
  uint8_t* shards;         // batch base (device)
  uint64_t* present;       // per-group presence masks (device, OR-ed)
  uint32_t* stats;         // accepted, bad flag, out of window, too short, duplicate (device, nullable)
  uint32_t* win;           // [groups][n] first packet index per (group, row) (k_rx_claim), or null
  uint32_t* dup;           // optimistic pass: set to 1 when a packet finds its presence bit set, or null
  const uint32_t* gate;    // if non-null, the kernel does nothing unless *gate != 0
  const uint64_t* prev;    // presence masks at call entry (launch_rx_begin's snapshot), or null: a packet
                           // whose bit was already set there is a duplicate of an earlier call's copy
  uint32_t fixup;          // re-place pass: claim winners only, no stats, presence already set
  const unsigned long long* seen;  // if non-null: k_rx_begin's record -- *seen >= call means some group had a
                           // presence bit set at call entry (or a concurrent later call's did); below
                           // call, none did, and the place pass skips its per-packet `prev` lookups
  unsigned long long call; // this call's id (per context, increasing)
  uint64_t npk;
  uint64_t slot;
  uint64_t first_group;
  uint64_t groups;
  uint64_t rstride;
  uint64_t gstride;
  uint32_t S;              // shard size (payload bytes kept per row)
  uint32_t n;              // d + p
  uint32_t frame;          // 1: frame rows -- the row holds packet bytes [0, S + 6), payload at column 6
  uint32_t fill;           // frame rows: bytes written per row (a multiple of 16 >= S + 6; zeros past S + 6)
};

// Claims every (group, row) for its first packet in ring order (atomicMin of
// the packet index into a.win, which launch_rx_fill sets to 0xffffffff), then
// places the winners.  a.win == null places every accepted packet.
// Call entry, one launch: *dup = 0, prev[g] = present[g], win[0 .. words) =
// 0xffffffff (claim words; win may be null), and atomicMax(seen, call) by
// every block that finds a presence bit set (seen may be null).
hipError_t launch_rx_begin(const uint64_t* present, uint64_t* prev, uint64_t groups, uint32_t* dup, uint32_t* win,
                           uint64_t words, unsigned long long* seen, unsigned long long call, hipStream_t s);
hipError_t launch_rx_fill(uint32_t* win, uint64_t words, const uint32_t* gate, hipStream_t s);
hipError_t launch_rx_claim(const RxArgs& a, hipStream_t s);
hipError_t launch_rx_scatter(const RxArgs& a, hipStream_t s);
// rows x [S bytes at src + r*spitch + off] -> dst + r*dpitch, zeros to round_up(S, 16)
// (src, spitch, dst, dpitch 16-B aligned; each src row readable to round_up(off + S, 16)).
hipError_t launch_shift_rows(const uint8_t* src, uint64_t spitch, uint32_t off, uint8_t* dst, uint64_t dpitch,
                             uint32_t S, uint64_t rows, hipStream_t s);

}  // namespace kern
}  // namespace ugo
