// fec.hpp -- C++ host mirror of jflyup/ugo's FEC object (ugo/fec.go), the
// caller of Encode/Reconstruct, over the MI355X engine.
//
// Same names, argument meaning and behaviour as the Go code:
//   newFEC    ugo/fec.go:45-72     nil (nullptr) on invalid geometry
//   decode    ugo/fec.go:78-89     header parse + copy into a pooled buffer
//   markData  ugo/fec.go:91-95     markFEC ugo/fec.go:97-104 (paws wrap)
//   input     ugo/fec.go:107-226   ordered rx queue, group detection, Reconstruct
//   calcECC   ugo/fec.go:228-243   Encode over data[k][offset:maxlen]
// sync.Pool (ugo/fec.go:26,67-69) is a LIFO free list of maxPacketSize
// buffers; like the Go pool, reused buffers keep stale tails (:84-87).
// currentMs (:73-75) is injectable for tests.
#pragma once
#include <cstddef>
#include <cstdint>
#include <functional>
#include <memory>
#include <vector>

#include "reedsolomon.hpp"

namespace ugo {

constexpr size_t fecHeaderSize = 6;       // ugo/constants.go:17
constexpr uint16_t typeData = 0xf1;       // :18
constexpr uint16_t typeFEC = 0xf2;        // :19
constexpr uint32_t fecExpire = 30000;     // :20 (ms)
constexpr size_t maxPacketSize = 1476;    // :29

struct fecPacket {
  uint32_t seqid = 0;
  uint16_t flag = 0;
  Bytes* data = nullptr;  // pooled buffer, len maxPacketSize
  uint32_t ts = 0;
  uint16_t Flag() const { return flag; }
  const Bytes& Data() const { return *data; }
};

uint32_t currentMs();

class FEC {
 public:
  static std::unique_ptr<FEC> newFEC(int rxlimit, int dataShards, int parityShards, int device = 0);

  fecPacket decode(const uint8_t* data, size_t len);
  void markData(uint8_t* data);
  void markFEC(uint8_t* data);
  // Returns the recovered data shards (index order); empty = Go's nil.
  std::vector<Bytes> input(fecPacket pkt);
  // Parity over data[k][offset:maxlen]; returns pointers to data[d:], or empty
  // on error (length mismatch, window outside a buffer, Encode error).
  std::vector<Bytes*> calcECC(std::vector<Bytes>& data, int offset, int maxlen);

  // Batched recovery (a GPU extension; ugo has none).  With setBatch(n), n > 0,
  // input() does not Reconstruct a recoverable lossy group itself
  // (ugo/fec.go:196-217): it copies the group's shards[k][:maxlen] into a
  // pinned group-major batch and recovers the whole batch in ONE launch when
  // it holds n groups (inside the input() call that completes it) or on
  // flush().  Recovered data shards come back group by group in completion
  // order, each group's in index order: exactly the concatenation of what
  // per-call input() returns, only later.  The rx queue, buffer pool, dedupe,
  // expiry and rxlimit trim do not change.  setBatch(0) restores the
  // reference's per-call behaviour.  Both return the shards of any groups
  // still pending (they are flushed first).  d+p must be <= 64.
  std::vector<Bytes> setBatch(int groups);
  std::vector<Bytes> flush();
  int batch() const { return batchCap_; }
  size_t pending() const { return pendMask_.size(); }
  ~FEC();

  // test / inspection hooks
  void setClock(std::function<uint32_t()> clock) { clock_ = std::move(clock); }
  size_t rxLen() const { return rx_.size(); }
  uint32_t next() const { return next_; }
  uint32_t paws() const { return paws_; }
  void setNext(uint32_t v) { next_ = v; }
  // a decoded packet that never reaches input() (bad flag, ugo/conn.go:395):
  // Go drops its pool buffer to the GC; so do we (it is never reused)
  void dropBuffer(Bytes* b);
  int dataShards() const { return dataShards_; }
  int parityShards() const { return parityShards_; }
  int lastError() const { return lastError_; }

 private:
  FEC() = default;
  Bytes* poolGet();
  void poolPut(Bytes* b);
  void recoverGroup(const std::vector<Bytes*>& shards, size_t maxlen, std::vector<Bytes>& out);
  void flushInto(std::vector<Bytes>& out);

  std::vector<fecPacket> rx_;  // ordered receive queue
  int rxlimit_ = 0;
  int dataShards_ = 0;
  int parityShards_ = 0;
  int shardSize_ = 0;
  uint32_t next_ = 0;
  std::unique_ptr<reedsolomon::Encoder> enc_;
  uint32_t paws_ = 0;
  uint32_t lastCheck_ = 0;
  std::vector<std::unique_ptr<Bytes>> poolAll_;
  std::vector<Bytes*> poolFree_;
  std::function<uint32_t()> clock_;
  int lastError_ = 0;
  // batched recovery: pinned [batchCap_][d+p][batchPitch_] and one presence
  // mask per pending group
  int batchCap_ = 0;
  size_t batchS_ = 0, batchPitch_ = 0, batchBytes_ = 0;
  uint8_t* batchBuf_ = nullptr;
  std::vector<uint64_t> pendMask_;
};

}  // namespace ugo
