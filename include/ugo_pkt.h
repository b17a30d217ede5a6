/*
 * ugo_pkt.h -- C-ABI of the batch decoder for ugo's packet wire format
 * (SURVEY.md §8f row 4), the step after FEC on the receive path:
 *
 *   Conn.handlePacket  ugo/conn.go:387-419   decrypt, FEC hook, strip the 6-B
 *                                            FEC header of typeData packets,
 *                                            then ugoPacket.decode
 *   ugoPacket.decode   ugo/packet.go:138-177 flags | SACK | packet number |
 *                                            stop-waiting | segments...
 *   parseSack          ugo/packet.go:231-331 (+ validateAckRanges :439-474)
 *   parseSegment       ugo/packet.go:78-100
 *   ReadUfloat16       ugo/utils/float16.go:25-51
 *
 * One call decodes a whole batch of received packets on the GPU (device
 * memory, stream-ordered).  Segment data is not copied: each segment reports
 * where its bytes sit in the packet (zero-copy view of the caller's buffer).
 */
#ifndef UGO_PKT_H
#define UGO_PKT_H

#include <stddef.h>
#include <stdint.h>

#include "ugo_fec.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Per-packet decode status: the error ugoPacket.decode would return. */
typedef enum ugo_pkt_status {
  UGO_PKT_OK = 0,
  UGO_PKT_EOF = 1,                     /* io.EOF */
  UGO_PKT_UNEXPECTED_EOF = 2,          /* io.ErrUnexpectedEOF */
  UGO_PKT_VARINT_OVERFLOW = 3,         /* "binary: varint overflows a 64-bit integer" */
  UGO_PKT_INVALID_ACK_RANGES = 4,      /* errInvalidAckRanges (ugo/packet.go:42) */
  UGO_PKT_INVALID_FIRST_ACK_RANGE = 5, /* errInvalidFirstAckRange (ugo/packet.go:44) */
  UGO_PKT_CAPACITY = 6                 /* decoded OK, but more ACK ranges / segments than the caller's arrays hold */
} ugo_pkt_status;

/* Decoded fixed fields of one packet (64 bytes). */
typedef struct ugo_pkt_info {
  uint64_t packet_number;    /* 0 for a pure ACK (flags == 0x80) */
  uint64_t stop_waiting;
  uint64_t largest_acked;    /* SACK fields: valid when flags & 0x80 */
  uint64_t largest_in_order;
  uint64_t delay_us;         /* ufloat16-decoded delay, microseconds */
  uint32_t status;           /* ugo_pkt_status */
  uint32_t payload_off;      /* where the ugoPacket starts in the slot (0, or 6 after a typeData FEC header) */
  uint16_t n_ranges;         /* ACK ranges stored in ranges[i*max_ranges ...] */
  uint16_t n_segments;       /* segments stored in segs[i*max_segments ...] */
  uint8_t flags;             /* ugoPacket flags byte */
  uint8_t fec_flag_lo;       /* low byte of the FEC header flag (framed mode), else 0 */
  uint8_t reserved[10];
} ugo_pkt_info;

/* One stream segment: offset uvarint, BE16 length, data. */
typedef struct ugo_pkt_segment {
  uint64_t offset;
  uint32_t data_off;  /* byte offset of the data within the slot */
  uint16_t len;       /* declared length = len(segment.data) */
  uint16_t avail;     /* bytes present; < len only for a truncated last segment,
                         whose remaining bytes read as zero (bytes.Reader.Read) */
} ugo_pkt_segment;

/* Framed mode: packets carry ugo's 6-B FEC header (FEC enabled).  As in
 * Conn.handlePacket, the header is stripped only for typeData (0xf1) packets;
 * every other packet is decoded from byte 0. */
#define UGO_PKT_FEC_FRAMED 1u

/* Decode npackets received packets: packet i is at pkts + i*slot (16-B aligned
 * slots), lens[i] bytes.  Buffers: device or pinned host memory (zero-copy,
 * as for ugo_fec_rx_assemble); pageable host memory is rejected.  pad (nullable, >= slot bytes) is XORed over each
 * packet from byte 0 first (the fixed-key RC4 Decrypt, ugo/conn.go:390).
 * info[npackets]; ranges[npackets][max_ranges][2] = {first, last} packet
 * numbers, highest range first; segs[npackets][max_segments].  A packet that
 * decodes without error but has more ranges or segments than the caps gets
 * UGO_PKT_CAPACITY (the first max_* are stored); a packet the reference would
 * reject gets the reference's error whatever its size.  Returns a
 * ugo_fec_status (argument / launch errors); per-packet results are in info. */
int ugo_fec_packet_decode(ugo_fec* ctx, const uint8_t* pkts, size_t slot, const uint16_t* lens, size_t npackets,
                          const uint8_t* pad, unsigned flags, ugo_pkt_info* info, uint64_t* ranges,
                          size_t max_ranges, ugo_pkt_segment* segs, size_t max_segments, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* UGO_PKT_H */
