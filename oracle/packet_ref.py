"""ORACLE -- TEST INFRASTRUCTURE ONLY: restatement of ugo's packet wire codec.

Only tests/ may import this module, as the checker for the batch decoder
(ugo_amd/csrc/pkt_kernels.hip, ugo_fec_packet_decode).  It restates:

  ugoPacket.decode     ugo/packet.go:138-177   flags, SACK, packet number,
                                               stop-waiting, segments until end
  parseSegment         ugo/packet.go:78-100    uvarint offset, BE16 length, data
                                               (bytes.Reader.Read: a short read
                                               is accepted, the tail stays zero)
  parseSack            ugo/packet.go:231-331   ACK ranges incl. long-gap blocks
  validateAckRanges    ugo/packet.go:439-474
  ReadUfloat16         ugo/utils/float16.go:25-51 (ReadUint16: utils.go:89-99, LE)
  binary.ReadUvarint   Go encoding/binary (standard library; the modern form
                       that stops after MaxVarintLen64 = 10 bytes)

and, to generate test packets, the encoder side:

  ugoPacket.encode     ugo/packet.go:185-229
  sack.write           ugo/packet.go:333-430 (delay is passed in: the reference
                       takes time.Now() - packetReceivedTime)
  segment.write        ugo/packet.go:102-111
  numWritableNackRanges ugo/packet.go:478-505
  WriteUfloat16        ugo/utils/float16.go:54-82

Error kinds are reported as the status codes of include/ugo_fec.h's packet
decoder (UGO_PKT_*).  Arithmetic on packet numbers wraps at 2^64 like Go's
uint64.
"""
from __future__ import annotations

M64 = (1 << 64) - 1

ackFlag, stopFlag, pshFlag, finFlag, rstFlag = 0x80, 0x40, 0x20, 0x10, 0x08

# status codes (include/ugo_fec.h, ugo_pkt_status)
PKT_OK = 0
PKT_EOF = 1              # io.EOF
PKT_UNEXPECTED_EOF = 2   # io.ErrUnexpectedEOF
PKT_VARINT_OVERFLOW = 3  # binary: varint overflows a 64-bit integer
PKT_INVALID_ACK_RANGES = 4
PKT_INVALID_FIRST_ACK_RANGE = 5


class DecodeError(Exception):
    def __init__(self, code):
        super().__init__(code)
        self.code = code


class EncodeError(Exception):
    pass


class Reader:
    """bytes.Reader over a packet."""

    def __init__(self, b: bytes):
        self.b = b
        self.i = 0

    def left(self):
        return len(self.b) - self.i

    def read_byte(self):
        if self.i >= len(self.b):
            raise DecodeError(PKT_EOF)
        v = self.b[self.i]
        self.i += 1
        return v

    def read_uvarint(self):
        x, s = 0, 0
        for i in range(10):
            if self.i >= len(self.b):
                raise DecodeError(PKT_UNEXPECTED_EOF if i > 0 else PKT_EOF)
            b = self.b[self.i]
            self.i += 1
            if b < 0x80:
                if i == 9 and b > 1:
                    raise DecodeError(PKT_VARINT_OVERFLOW)
                return (x | (b << s)) & M64
            x |= (b & 0x7F) << s
            s += 7
        raise DecodeError(PKT_VARINT_OVERFLOW)

    def read_be16(self):  # binary.Read(r, BigEndian, &uint16): io.ReadFull
        n = self.left()
        if n == 0:
            raise DecodeError(PKT_EOF)
        if n == 1:
            self.i += 1
            raise DecodeError(PKT_UNEXPECTED_EOF)
        v = (self.b[self.i] << 8) | self.b[self.i + 1]
        self.i += 2
        return v

    def read_ufloat16(self):
        b1 = self.read_byte()
        b2 = self.read_byte()
        val = b1 | (b2 << 8)
        if val < (1 << 12):
            return val
        exponent = (val >> 11) - 1
        res = val - (exponent << 11)
        return (res << exponent) & M64


def parse_sack(r: Reader):
    type_byte = r.read_byte()
    has_missing = (type_byte & 0x20) == 0x20
    largest = r.read_uvarint()
    delay = r.read_ufloat16()
    num_blocks = 0
    if has_missing:
        num_blocks = r.read_byte()
    if has_missing and num_blocks == 0:
        raise DecodeError(PKT_INVALID_ACK_RANGES)
    blen = r.read_uvarint()
    if blen < 1:
        raise DecodeError(PKT_INVALID_FIRST_ACK_RANGE)
    if blen > largest:
        raise DecodeError(PKT_INVALID_ACK_RANGES)
    ranges = []
    if has_missing:
        ranges.append([(largest - blen + 1) & M64, largest])
        in_long = False
        last_complete = False
        for _ in range(num_blocks):
            gap = r.read_byte()
            blen = r.read_uvarint()
            if in_long:
                ranges[-1][0] = (ranges[-1][0] - (gap + blen)) & M64
                ranges[-1][1] = (ranges[-1][1] - gap) & M64
            else:
                last_complete = False
                last = (ranges[-1][0] - gap - 1) & M64
                ranges.append([(last - blen + 1) & M64, last])
            if blen > 0:
                last_complete = True
            in_long = blen == 0
        if not last_complete:
            ranges.pop()
        in_order = ranges[-1][0]
    else:
        in_order = (largest + 1 - blen) & M64
    # validateAckRanges
    if ranges:
        ok = len(ranges) != 1 and ranges[0][1] == largest
        ok = ok and all(f <= l for f, l in ranges)
        for i in range(1, len(ranges)):
            if not ok:
                break
            if ranges[i - 1][0] <= ranges[i][0] or ranges[i - 1][0] <= (ranges[i][1] + 1) & M64:
                ok = False
        if not ok:
            raise DecodeError(PKT_INVALID_ACK_RANGES)
    return {"largest_acked": largest, "largest_in_order": in_order, "delay_us": delay,
            "ranges": [tuple(x) for x in ranges]}


def decode(raw: bytes):
    """ugoPacket.decode.  Returns (status, fields): on error the fields parsed
    so far are irrelevant (conn.go:416-419 drops the packet)."""
    r = Reader(raw)
    out = {"flags": 0, "sack": None, "packet_number": 0, "stop_waiting": 0, "segments": []}
    try:
        out["flags"] = flags = r.read_byte()
        if flags & ackFlag:
            out["sack"] = parse_sack(r)
        if flags != ackFlag:
            out["packet_number"] = r.read_uvarint()
        if flags & stopFlag:
            out["stop_waiting"] = r.read_uvarint()
        while r.left() > 0:
            off = r.read_uvarint()
            n = r.read_be16()
            start = r.i
            avail = 0
            if n != 0:
                if r.left() == 0:
                    raise DecodeError(PKT_EOF)  # bytes.Reader.Read at end
                avail = min(n, r.left())
                r.i += avail
            out["segments"].append((off, start, n, avail))
    except DecodeError as e:
        return e.code, out
    return PKT_OK, out


# ------------------------------------------------------------------ encoder
def put_uvarint(v: int) -> bytes:
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def write_ufloat16(value: int) -> bytes:
    if value < (1 << 12):
        res = value
    elif value >= ((1 << 12) - 1) << 30:
        res = 0xFFFF
    else:
        exponent = 0
        offset = 16
        while offset > 0:
            if value >= (1 << (11 + offset)):
                exponent += offset
                value >>= offset
            offset //= 2
        res = (value + (exponent << 11)) & 0xFFFF
    return bytes([res & 0xFF, res >> 8])


def _num_writable_nack_ranges(ranges):
    if not ranges:
        return 0
    num = 0
    for i in range(1, len(ranges)):
        gap = (ranges[i - 1][0] - ranges[i][1]) & M64
        rl = gap // 256 + (1 if gap % 256 else 0)
        if num + rl < 0xFF:
            num += rl
        else:
            break
    return num + 1


def write_sack(largest, in_order, ranges, delay_us) -> bytes:
    b = bytearray()
    has_missing = len(ranges) > 0
    b.append(0x20 if has_missing else 0)
    b += put_uvarint(largest)
    b += write_ufloat16(delay_us)
    num_ranges = written = 0
    if has_missing:
        num_ranges = _num_writable_nack_ranges(ranges)
        assert num_ranges <= 0xFF
        b.append((num_ranges - 1) & 0xFF)
        first_len = largest - ranges[0][0] + 1
        written += 1
    else:
        first_len = largest - in_order + 1
    b += put_uvarint(first_len)
    for i in range(1, len(ranges)):
        length = ranges[i][1] - ranges[i][0] + 1
        gap = ranges[i - 1][0] - ranges[i][1] - 1
        num = gap // 0xFF + 1
        if gap % 0xFF == 0:
            num -= 1
        if num == 1:
            b.append(gap & 0xFF)
            b += put_uvarint(length)
            written += 1
        else:
            for j in range(num):
                if j == num - 1:
                    b.append(gap % 0xFF)
                    b += put_uvarint(length)
                else:
                    b.append(0xFF)
                    b += put_uvarint(0)
                written += 1
        if written >= num_ranges:
            break
    if num_ranges != written:
        # ugo/packet.go:414-416: numWritableNackRanges counts gap/256 blocks, the
        # writer gap-1 / 255, so some long gaps (e.g. 767) disagree and encode()
        # fails ("BUG: Inconsistent number of ACK ranges written"): never sent
        raise EncodeError("inconsistent number of ACK ranges written")
    return bytes(b)


def encode(flags=0, sack=None, packet_number=0, stop_waiting=0, segments=()):
    """ugoPacket.encode; sack = (largest, in_order, ranges, delay_us) or None,
    segments = [(offset, data_bytes)]."""
    if sack is not None:
        flags |= ackFlag
    if stop_waiting != 0:
        flags |= stopFlag
    if segments:
        flags |= pshFlag
    b = bytearray([flags])
    if sack is not None:
        b += write_sack(*sack)
    if flags != ackFlag:
        b += put_uvarint(packet_number)
    if stop_waiting != 0:
        b += put_uvarint(stop_waiting)
    for off, data in segments:
        b += put_uvarint(off)
        b += bytes([(len(data) >> 8) & 0xFF, len(data) & 0xFF])
        b += data
    return bytes(b)
