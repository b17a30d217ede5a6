// pkt_kernels.hip -- batch decoder for ugo's packet wire format on gfx950
// (SURVEY.md §8f row 4).  One thread per packet restates, for a whole batch:
//   Conn.handlePacket  ugo/conn.go:387-419  decrypt, strip the FEC header of
//                                           typeData packets, ugoPacket.decode
//   ugoPacket.decode   ugo/packet.go:138-177
//   parseSack          ugo/packet.go:231-331, validateAckRanges :439-474
//   parseSegment       ugo/packet.go:78-100
//   ReadUfloat16       ugo/utils/float16.go:25-51, binary.ReadUvarint (Go stdlib)
//
// The parse is serial within a packet (varints, data-dependent skips), so the
// parallelism is across packets.  Bytes are read through a 16-byte window
// held in registers (one aligned dwordx4 load, plus the pad chunk when
// decrypting, per 16 bytes touched): a typical data packet touches only its
// first window and the window of its segment header; segment data is never
// read -- segments are reported as (offset, data_off, len, avail) views.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "launch.hpp"
#include "pkt_kernels.hpp"

namespace ugo {
namespace kern {

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct ByteReader {
  const uint8_t* base;  // slot start
  const uint8_t* pad;
  uint32_t pos, end;
  uint32_t wchunk;      // 16-B chunk index held in w (~0u: none)
  u32x4 w;

  __device__ __forceinline__ uint32_t byte_at(uint32_t j) {
    if ((j >> 4) != wchunk) {
      wchunk = j >> 4;
      w = *reinterpret_cast<const u32x4*>(base + (j & ~15u));
      if (pad) w ^= *reinterpret_cast<const u32x4*>(pad + (j & ~15u));
    }
    const uint32_t q = (j >> 2) & 3u;
    const uint32_t d = (q & 2u) ? ((q & 1u) ? w.w : w.z) : ((q & 1u) ? w.y : w.x);
    return (d >> (8u * (j & 3u))) & 0xffu;
  }
  __device__ __forceinline__ uint32_t left() const { return end - pos; }
};

enum : uint32_t {
  kOK = UGO_PKT_OK,
  kEOF = UGO_PKT_EOF,
  kUnexpectedEOF = UGO_PKT_UNEXPECTED_EOF,
  kOverflow = UGO_PKT_VARINT_OVERFLOW,
  kInvalidRanges = UGO_PKT_INVALID_ACK_RANGES,
  kInvalidFirst = UGO_PKT_INVALID_FIRST_ACK_RANGE,
  kCapacity = UGO_PKT_CAPACITY,
};

__device__ __forceinline__ uint32_t read_byte(ByteReader& r, uint32_t& v) {
  if (r.pos >= r.end) return kEOF;
  v = r.byte_at(r.pos++);
  return kOK;
}

// binary.ReadUvarint (at most MaxVarintLen64 = 10 bytes)
__device__ __forceinline__ uint32_t read_uvarint(ByteReader& r, uint64_t& x) {
  x = 0;
  uint32_t s = 0;
  for (int i = 0; i < 10; ++i) {
    if (r.pos >= r.end) return i > 0 ? kUnexpectedEOF : kEOF;
    const uint32_t b = r.byte_at(r.pos++);
    if (b < 0x80u) {
      if (i == 9 && b > 1u) return kOverflow;
      x |= static_cast<uint64_t>(b) << s;
      return kOK;
    }
    x |= static_cast<uint64_t>(b & 0x7fu) << s;
    s += 7;
  }
  return kOverflow;
}

// ReadUfloat16: utils.ReadUint16 (two ReadByte, little endian) + decode
__device__ __forceinline__ uint32_t read_ufloat16(ByteReader& r, uint64_t& v) {
  uint32_t b1, b2;
  uint32_t st = read_byte(r, b1);
  if (st) return st;
  st = read_byte(r, b2);
  if (st) return st;
  const uint32_t val = b1 | (b2 << 8);
  if (val < (1u << 12)) {
    v = val;
    return kOK;
  }
  const uint32_t exponent = (val >> 11) - 1u;
  v = static_cast<uint64_t>(val - (exponent << 11)) << exponent;
  return kOK;
}

// parseSack + validateAckRanges, streaming: a range is final once the next
// one starts (only the last range is ever modified or dropped, ugo/packet.go:
// 285-306), so it is validated against its predecessor and stored then.
// Ranges beyond the caller's cap are validated but not stored (`over`).
// Returns a hard error, or OK with `over` telling whether ranges were dropped.
__device__ uint32_t parse_sack(ByteReader& r, ugo_pkt_info& o, uint64_t* rg, uint32_t cap, bool& over) {
  uint32_t type_byte;
  uint32_t st = read_byte(r, type_byte);
  if (st) return st;
  const bool has_missing = (type_byte & 0x20u) != 0;
  uint64_t largest;
  if ((st = read_uvarint(r, largest))) return st;
  o.largest_acked = largest;
  uint64_t delay;
  if ((st = read_ufloat16(r, delay))) return st;
  o.delay_us = delay;
  uint32_t nblocks = 0;
  if (has_missing && (st = read_byte(r, nblocks))) return st;
  if (has_missing && nblocks == 0) return kInvalidRanges;
  uint64_t blen;
  if ((st = read_uvarint(r, blen))) return st;
  if (blen < 1) return kInvalidFirst;
  if (blen > largest) return kInvalidRanges;
  if (!has_missing) {
    o.largest_in_order = largest + 1 - blen;
    return kOK;
  }
  uint64_t cf = largest - blen + 1, cl = largest;  // current (last) range
  uint64_t pf = 0;                                  // first of the last final range
  uint32_t nfinal = 0;
  bool invalid = false;
  auto finalize = [&](uint64_t f, uint64_t l) {
    if (f > l) invalid = true;
    if (nfinal > 0 && (pf <= f || pf <= l + 1)) invalid = true;
    if (nfinal < cap) {
      rg[2 * nfinal] = f;
      rg[2 * nfinal + 1] = l;
    } else {
      over = true;
    }
    pf = f;
    ++nfinal;
  };
  bool in_long = false, last_complete = false;
  for (uint32_t i = 0; i < nblocks; ++i) {
    uint32_t gap;
    if ((st = read_byte(r, gap))) return st;
    if ((st = read_uvarint(r, blen))) return st;
    if (in_long) {
      cf -= static_cast<uint64_t>(gap) + blen;
      cl -= gap;
    } else {
      last_complete = false;
      finalize(cf, cl);
      cl = cf - gap - 1;
      cf = cl - blen + 1;
    }
    if (blen > 0) last_complete = true;
    in_long = blen == 0;
  }
  if (last_complete) finalize(cf, cl);  // else the last range is dropped
  o.n_ranges = static_cast<uint16_t>(min(nfinal, cap));
  o.largest_in_order = pf;
  // validateAckRanges: >= 2 ranges; range 0 ends at largest (it is never
  // modified after it is final, so this holds by construction)
  if (nfinal == 1 || invalid) return kInvalidRanges;
  return kOK;
}

__device__ uint32_t decode_one(ByteReader& r, ugo_pkt_info& o, uint64_t* rg, uint32_t rcap, ugo_pkt_segment* sg,
                               uint32_t scap) {
  uint32_t flags;
  uint32_t st = read_byte(r, flags);
  if (st) return st;
  o.flags = static_cast<uint8_t>(flags);
  bool over = false;  // more ranges / segments than the caller's arrays hold
  if (flags & 0x80u) {
    st = parse_sack(r, o, rg, rcap, over);
    if (st) return st;
  }
  if (flags != 0x80u && (st = read_uvarint(r, o.packet_number))) return st;
  if ((flags & 0x40u) && (st = read_uvarint(r, o.stop_waiting))) return st;
  uint32_t ns = 0;
  while (r.left() > 0) {
    uint64_t off;
    if ((st = read_uvarint(r, off))) return st;
    // binary.Read(r, BigEndian, &uint16): io.ReadFull of 2 bytes
    if (r.left() == 0) return kEOF;
    if (r.left() == 1) return kUnexpectedEOF;
    const uint32_t len = (r.byte_at(r.pos) << 8) | r.byte_at(r.pos + 1);
    r.pos += 2;
    uint32_t avail = 0;
    const uint32_t data_off = r.pos;
    if (len != 0) {
      if (r.left() == 0) return kEOF;  // bytes.Reader.Read at the end
      avail = min(len, r.left());
      r.pos += avail;
    }
    if (ns < scap) {
      sg[ns] = ugo_pkt_segment{off, data_off, static_cast<uint16_t>(len), static_cast<uint16_t>(avail)};
      o.n_segments = static_cast<uint16_t>(ns + 1);
    } else {
      over = true;
    }
    ++ns;
  }
  return over ? kCapacity : kOK;
}

__global__ __launch_bounds__(256) void k_packet_decode(PktArgs a) {
  const uint64_t i = blockIdx.x * 256ull + threadIdx.x;
  if (i >= a.npk) return;
  ByteReader r;
  r.base = a.pkts + i * a.slot;
  r.pad = a.pad;
  r.end = min(static_cast<uint32_t>(a.lens[i]), static_cast<uint32_t>(a.slot));
  r.pos = 0;
  r.wchunk = ~0u;
  r.w = u32x4{0u, 0u, 0u, 0u};
  ugo_pkt_info o{};
  if (a.framed && r.end >= 6u) {
    const uint32_t flag = r.byte_at(4) | (r.byte_at(5) << 8);  // FEC.decode, ugo/fec.go:81
    o.fec_flag_lo = static_cast<uint8_t>(flag);
    if (flag == 0xf1u) r.pos = 6;  // typeData: data = data[fecHeaderSize:] (ugo/conn.go:403-405)
  }
  o.payload_off = r.pos;
  o.status = decode_one(r, o, a.ranges + i * 2ull * a.max_ranges, a.max_ranges, a.segs + i * a.max_segments,
                        a.max_segments);
  a.info[i] = o;
}

}  // namespace

hipError_t launch_packet_decode(const PktArgs& a, hipStream_t s) {
  if (a.npk == 0) return hipSuccess;
  const uint64_t blocks = (a.npk + 255) / 256;
  launch(kKPacket, k_packet_decode, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace kern
}  // namespace ugo
