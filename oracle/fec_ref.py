"""ORACLE -- TEST INFRASTRUCTURE ONLY: pure-Python restatement of ugo/fec.go.

Only tests/ may import this module, as the checker for the C++ host mirror
(ugo_amd/csrc/host/fec.cpp).  It restates, line by line in behaviour:

  newFEC     ugo/fec.go:45-72    geometry checks, paws = (0xffffffff/n - 1)*n
  decode     ugo/fec.go:78-89    LE32 seqid, LE16 flag, ts, copy data[6:] into a pooled
                                 maxPacketSize buffer (stale tail kept, :84-87)
  markData   ugo/fec.go:91-95    LE32 next, LE16 typeData, next++
  markFEC    ugo/fec.go:97-104   LE32 next, LE16 typeFEC, next++, wrap at paws
  input      ugo/fec.go:107-226  expiry sweep, ordered insert + dedupe, group window
                                 search, no-loss release, Reconstruct, rxlimit trim
  calcECC    ugo/fec.go:228-243  Encode over data[k][offset:maxlen]
  tx_group   ugo/conn.go:643-685 the sender loop (markData, copy, calcECC(.., 6,
                                 maxsize), markFEC, ecc[k][:maxsize]) for one group,
                                 then crypt.Encrypt (ugo/conn.go:634) per packet

Go's sync.Pool (ugo/fec.go:26, :67-69) is modelled as a LIFO free list (the
C++ mirror uses the same discipline), so stale-tail bytes are deterministic.
Reed-Solomon arithmetic comes from the C oracle (rs_ref.c_encode /
c_reconstruct), i.e. the upstream klauspost restatement.
"""
from __future__ import annotations

import struct

import numpy as np

import rs_ref

fecHeaderSize = 6  # ugo/constants.go:17
typeData = 0xF1    # :18
typeFEC = 0xF2     # :19
fecExpire = 30000  # :20 (ms)
maxPacketSize = 1476  # :29


class Pool:
    """LIFO model of fec.xmitBuf (sync.Pool with New = make([]byte, maxPacketSize))."""

    def __init__(self):
        self.free = []

    def get(self):
        return self.free.pop() if self.free else bytearray(maxPacketSize)

    def put(self, b):
        self.free.append(b)


class Packet:
    __slots__ = ("seqid", "flag", "data", "ts")

    def __init__(self, seqid, flag, data, ts):
        self.seqid, self.flag, self.data, self.ts = seqid, flag, data, ts


class FEC:
    def __init__(self, rxlimit, d, p, clock):
        self.rx = []
        self.rxlimit = rxlimit
        self.dataShards = d
        self.parityShards = p
        self.shardSize = d + p
        self.next = 0
        self.paws = ((0xFFFFFFFF // self.shardSize) - 1) * self.shardSize
        self.lastCheck = 0
        self.pool = Pool()
        self.clock = clock

    @staticmethod
    def new(rxlimit, d, p, clock):
        if d <= 0 or p <= 0:
            return None
        if rxlimit < d + p:
            return None
        return FEC(rxlimit, d, p, clock)

    def decode(self, data: bytes) -> Packet:
        seqid, flag = struct.unpack_from("<IH", data, 0)
        buf = self.pool.get()
        payload = data[6:]
        n = min(len(buf), len(payload))
        buf[:n] = payload[:n]
        return Packet(seqid, flag, buf, self.clock() & 0xFFFFFFFF)

    def markData(self, data: bytearray):
        struct.pack_into("<IH", data, 0, self.next, typeData)
        self.next = (self.next + 1) & 0xFFFFFFFF

    def markFEC(self, data: bytearray):
        struct.pack_into("<IH", data, 0, self.next, typeFEC)
        self.next = (self.next + 1) & 0xFFFFFFFF
        if self.next >= self.paws:
            self.next = 0

    def input(self, pkt: Packet):
        recovered = None
        now = self.clock() & 0xFFFFFFFF
        if ((now - self.lastCheck) & 0xFFFFFFFF) >= fecExpire:
            keep = []
            for q in self.rx:
                if ((now - q.ts) & 0xFFFFFFFF) < fecExpire:
                    keep.append(q)
                else:
                    self.pool.put(q.data)
            self.rx = keep
            self.lastCheck = now
        n = len(self.rx) - 1
        insertIdx = 0
        for i in range(n, -1, -1):
            if pkt.seqid == self.rx[i].seqid:
                self.pool.put(pkt.data)
                return None
            elif pkt.seqid > self.rx[i].seqid:
                insertIdx = i + 1
                break
        self.rx.insert(insertIdx, pkt)
        shardBegin = pkt.seqid - pkt.seqid % self.shardSize
        shardEnd = (shardBegin + self.shardSize - 1) & 0xFFFFFFFF
        searchBegin = max(insertIdx - self.shardSize, 0)
        searchEnd = insertIdx + self.shardSize
        if searchEnd >= len(self.rx):
            searchEnd = len(self.rx) - 1
        if len(self.rx) >= self.dataShards and shardBegin < shardEnd:
            numshard = numDataShard = 0
            first = -1
            maxlen = 0
            shards = [None] * self.shardSize
            flags = [False] * self.shardSize
            for i in range(searchBegin, searchEnd + 1):
                seqid = self.rx[i].seqid
                if seqid > shardEnd:
                    break
                elif seqid >= shardBegin:
                    shards[seqid % self.shardSize] = self.rx[i].data
                    flags[seqid % self.shardSize] = True
                    numshard += 1
                    if self.rx[i].flag == typeData:
                        numDataShard += 1
                    if numshard == 1:
                        first = i
                    maxlen = max(maxlen, len(self.rx[i].data))
            if numDataShard == self.dataShards:
                for i in range(first, first + numshard):
                    self.pool.put(self.rx[i].data)
                del self.rx[first:first + numshard]
            elif numshard >= self.dataShards:
                recovered = self._reconstruct(shards, flags, maxlen)
                for i in range(first, first + numshard):
                    self.pool.put(self.rx[i].data)
                del self.rx[first:first + numshard]
        if len(self.rx) > self.rxlimit:
            self.pool.put(self.rx[0].data)
            self.rx = self.rx[1:]
        return recovered

    def _reconstruct(self, shards, flags, maxlen):
        n, d = self.shardSize, self.dataShards
        grp = np.zeros((1, n, maxlen), np.uint8)
        mask = 0
        for k in range(n):
            if shards[k] is not None:
                grp[0, k] = np.frombuffer(bytes(shards[k][:maxlen]), np.uint8)
                mask |= 1 << k
        rc, st = rs_ref.c_reconstruct(d, self.parityShards, grp, np.array([mask], np.uint64))
        if rc:
            return None  # error logged and swallowed (ugo/fec.go:208-210)
        out = [bytearray(grp[0, k].tobytes()) for k in range(d) if not flags[k]]
        return out or None

    def calcECC(self, data, offset, maxlen):
        if len(data) != self.shardSize:
            return None
        n, d = self.shardSize, self.dataShards
        S = maxlen - offset
        if S <= 0:
            return None  # Encode: ErrShardNoData
        grp = np.zeros((1, n, S), np.uint8)
        for k in range(d):
            grp[0, k] = np.frombuffer(bytes(data[k][offset:maxlen]), np.uint8)
        rs_ref.c_encode(d, self.parityShards, grp)
        for k in range(d, n):
            data[k][offset:maxlen] = grp[0, k].tobytes()
        return data[d:]


def handle(fec: FEC, wire: bytes):
    """Conn.handlePacket's FEC hook (ugo/conn.go:394-396): decode, then input()
    only for typeData / typeFEC packets (other buffers are dropped, never Put)."""
    pkt = fec.decode(wire)
    rec = None
    if pkt.flag in (typeData, typeFEC):
        rec = fec.input(pkt)
    return pkt.seqid, pkt.flag, rec


def tx_group(fec: FEC, data_pkts, key=None, buf_size=maxPacketSize):
    """One group of the sender loop ugo/conn.go:643-685 on FRESH, zero-filled
    group buffers (the reference reuses its 13 buffers without clearing them, so
    its parity bytes past a short packet's end depend on earlier groups; the
    batch TX contract is the fresh-buffer result), followed by the fixed-key
    RC4 encryption of every wire packet (ugo/conn.go:634, ugo/crypto.go:33-39).
    Returns the d + p wire packets in send order."""
    import rc4_ref
    d, n = fec.dataShards, fec.shardSize
    group = [bytearray(max(buf_size, max(len(x) for x in data_pkts))) for _ in range(n)]
    out, maxsize = [], 0
    for k, ori in enumerate(data_pkts):
        ori = bytearray(ori)
        fec.markData(ori)
        group[k][:len(ori)] = ori
        maxsize = max(maxsize, len(ori))
        out.append(bytes(ori))
    ecc = fec.calcECC(group, fecHeaderSize, maxsize)
    # calcECC returns nil when Encode fails (every packet header-only: empty
    # window, ErrShardNoData): the loop then sends no parity (ugo/conn.go:669-673)
    for k in range(len(ecc) if ecc is not None else 0):
        fec.markFEC(ecc[k])
        out.append(bytes(ecc[k][:maxsize]))
    if key is not None:
        out = [rc4_ref.xor_stream(key, w) for w in out]
    return out
