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
//
// The pool lives in pinned host memory (slabs of 16-B aligned slots), so a
// lost group's survivors are read by the GPU where decode put them
// (ugo_fec_reconstruct_rows): no copy into a batch.  A pool buffer is a
// logical buffer over a physical slot.  The logical buffers keep the Go
// pool's LIFO order and bytes exactly; when a buffer whose slot a pending
// batch still has to read is reused, the buffer moves to a fresh slot first,
// carrying its stale tail (decode overwrites only the head), and the old slot
// is freed once that batch is recovered.
#pragma once
#include <hip/hip_runtime_api.h>

#include <algorithm>
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
constexpr size_t kSlotStride = (maxPacketSize + 15) / 16 * 16;  // 1488: 16-B aligned slots

// One buffer of the Go pool ([]byte of len maxPacketSize): its bytes are the
// physical slot `slot` of the FEC's pinned slabs.
struct PoolBuf {
  uint32_t slot = 0;
};

struct fecPacket {
  uint32_t seqid = 0;
  uint16_t flag = 0;
  PoolBuf* data = nullptr;  // pooled buffer, len maxPacketSize
  uint32_t ts = 0;
  uint16_t Flag() const { return flag; }
};

uint32_t currentMs();

// Batched recovery flag (include/ugo_fec_conn.h UGO_FECCONN_BATCH_OVERLAP).
constexpr unsigned kBatchOverlap = 1u;

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
  // The same over n caller buffers of lengths lens[] (the C-ABI's form: no
  // copies of the packets), parity into bufs[d..n)[offset:maxlen); a status.
  int calcECC(uint8_t* const* bufs, const size_t* lens, int n, int offset, int maxlen);

  // Batched recovery (a GPU extension; ugo has none).  With setBatch(n), n > 0,
  // input() does not Reconstruct a recoverable lossy group itself
  // (ugo/fec.go:196-217): it records the group (its survivors' pool slots and
  // presence mask) and recovers the whole batch in ONE launch when it holds
  // n groups, or on flush().  Recovered data shards come back group by group
  // in completion order, each group's in index order: exactly the
  // concatenation of what per-call input() returns, only later.
  //   flags 0: the batch is recovered inside the input() call that fills it;
  //   kBatchOverlap: that launch runs while input() goes on with the next
  //     batch, and its shards come back from the input() call that fills the
  //     NEXT batch (or from flush()) -- one batch later, the GPU time hidden.
  // The rx queue, buffer pool, dedupe, expiry and rxlimit trim do not change.
  // setBatch(0) restores the reference's per-call behaviour.  Both return the
  // shards of any groups still pending (they are flushed first).  d+p <= 64.
  std::vector<Bytes> setBatch(int groups, unsigned flags = 0);
  std::vector<Bytes> flush();
  int batch() const { return batchCap_; }
  unsigned batchFlags() const { return batchFlags_; }
  // most groups one input() / flush() can return in the current mode
  size_t maxReturnGroups(bool isFlush) const;
  size_t pending() const;
  // Per-call latency service on this object's encoder (ugo_fec_service_start):
  // calcECC's Encode and per-call recovery's Reconstruct are then served by a
  // resident workgroup instead of a launch each.  idle_us < 0 stops it.
  int service(int idle_us);
  ~FEC();

  // test / inspection hooks
  void setClock(std::function<uint32_t()> clock) { clock_ = std::move(clock); }
  size_t rxLen() const { return rx_.size(); }
  uint32_t next() const { return next_; }
  uint32_t paws() const { return paws_; }
  void setNext(uint32_t v) { next_ = v; }
  // a decoded packet that never reaches input() (bad flag, ugo/conn.go:395):
  // Go drops its pool buffer to the GC; so do we (it is never reused)
  void dropBuffer(PoolBuf* b);
  int dataShards() const { return dataShards_; }
  int parityShards() const { return parityShards_; }
  int lastError() const { return lastError_; }
  const uint8_t* bytes(const PoolBuf* b) const { return slotPtr_[b->slot]; }

 private:
  // One pinned batch of staged lossy groups: row-pointer table, presence
  // masks, statuses and the recovered rows, plus the pool slots it reads.
  struct Batch {
    uint8_t* mem = nullptr;
    size_t cap = 0;
    uint64_t* rows = nullptr;  // [cap][n] device addresses
    uint64_t* masks = nullptr; // [cap]
    int8_t* status = nullptr;  // [cap]
    uint8_t* out = nullptr;    // [cap][min(d, p)][kSlotStride]: erased data rows, ascending
    size_t groups = 0;
    size_t S = 0;
    std::vector<uint32_t> held;
    hipEvent_t done = nullptr;
    bool inflight = false;
    int err = 0;  // status of its launch
  };

  FEC() = default;
  // recovered rows per staged group: a recoverable group misses at most min(d, p) data rows
  size_t outSlots() const { return static_cast<size_t>(std::min(dataShards_, parityShards_)); }
  PoolBuf* poolGet();
  void poolPut(PoolBuf* b);
  uint32_t newSlot(bool zero);
  uint8_t* writable(PoolBuf* b, size_t n);
  void releaseSlot(uint32_t s);
  bool ensureGpu();
  bool ensureBatch(Batch& b, size_t cap);
  void freeBatch(Batch& b);
  void recoverGroup(const std::vector<PoolBuf*>& shards, size_t maxlen, std::vector<Bytes>& out);
  bool recoverOne(const std::vector<PoolBuf*>& shards, size_t maxlen, std::vector<Bytes>& out);
  bool stage(Batch& b, const std::vector<PoolBuf*>& shards, size_t maxlen);
  bool launch(Batch& b);
  void collect(Batch& b, std::vector<Bytes>& out);
  void launchCurrent(std::vector<Bytes>& out);
  void flushInto(std::vector<Bytes>& out);

  std::vector<fecPacket> rx_;  // ordered receive queue
  int rxlimit_ = 0;
  int dataShards_ = 0;
  int parityShards_ = 0;
  int shardSize_ = 0;
  int device_ = 0;
  uint32_t next_ = 0;
  std::unique_ptr<reedsolomon::Encoder> enc_;
  uint32_t paws_ = 0;
  uint32_t lastCheck_ = 0;
  // pool: logical buffers (LIFO free list, as sync.Pool) over physical slots
  std::vector<std::unique_ptr<PoolBuf>> poolAll_;
  std::vector<PoolBuf*> poolFree_;
  std::vector<uint8_t*> slabs_;
  std::vector<uint8_t> slabPinned_;
  std::vector<uint8_t*> slotPtr_;
  std::vector<uint64_t> slotDev_;   // device address (0: slot not GPU-visible)
  std::vector<uint8_t> slotHeld_;   // a pending / in-flight batch reads this slot
  std::vector<uint8_t> slotOrphan_; // its buffer moved on or was dropped: free when unheld
  std::vector<uint32_t> slotFree_;
  std::function<uint32_t()> clock_;
  int lastError_ = 0;
  // recovery on the GPU: one stream for the batches; per call a pinned
  // one-group stage (recoverOne)
  hipStream_t stream_ = nullptr;
  uint8_t* one_ = nullptr;
  size_t oneBytes_ = 0;
  int batchCap_ = 0;
  unsigned batchFlags_ = 0;
  Batch batch_[2];
  int cur_ = 0;
};

}  // namespace ugo
