// fec.cpp -- see fec.hpp.  Control logic mirrors ugo/fec.go line by line in
// behaviour; every byte of Reed-Solomon arithmetic runs on the GPU through
// the C-ABI (ugo_fec_reconstruct_rows over the pinned pool, reedsolomon::
// Encoder for calcECC), none on the CPU.
#include "fec.hpp"

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>

namespace ugo {

namespace {

constexpr size_t kSlabSlots = 256;  // pool slots per pinned slab (372 KiB)

struct DevGuard {
  int prev = -1;
  explicit DevGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DevGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

}  // namespace

uint32_t currentMs() {  // ugo/fec.go:73-75
  using namespace std::chrono;
  return static_cast<uint32_t>(duration_cast<milliseconds>(system_clock::now().time_since_epoch()).count());
}

static inline void putLE32(uint8_t* p, uint32_t v) {
  p[0] = uint8_t(v); p[1] = uint8_t(v >> 8); p[2] = uint8_t(v >> 16); p[3] = uint8_t(v >> 24);
}
static inline void putLE16(uint8_t* p, uint16_t v) { p[0] = uint8_t(v); p[1] = uint8_t(v >> 8); }
static inline uint32_t getLE32(const uint8_t* p) {
  return uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24;
}
static inline uint16_t getLE16(const uint8_t* p) { return uint16_t(p[0] | p[1] << 8); }

std::unique_ptr<FEC> FEC::newFEC(int rxlimit, int dataShards, int parityShards, int device) {
  if (dataShards <= 0 || parityShards <= 0) return nullptr;  // :46-48
  if (rxlimit < dataShards + parityShards) return nullptr;  // :49-51
  std::unique_ptr<FEC> f(new FEC());
  f->rxlimit_ = rxlimit;
  f->dataShards_ = dataShards;
  f->parityShards_ = parityShards;
  f->shardSize_ = dataShards + parityShards;
  f->device_ = device;
  f->paws_ = (0xffffffffu / uint32_t(f->shardSize_) - 1) * uint32_t(f->shardSize_);  // :58
  int err = 0;
  f->enc_ = reedsolomon::New(dataShards, parityShards, &err, device);  // :59
  if (!f->enc_) return nullptr;  // :60-63 (logged upstream)
  f->clock_ = currentMs;
  return f;
}

// ------------------------------------------------------------------- pool

// A physical slot: from the free list, else a new slab.  Pinned slabs are
// GPU-visible (slotDev_ != 0); if pinned memory runs out, plain memory keeps
// the pool working and lost groups then recover through copies (recoverGroup).
uint32_t FEC::newSlot(bool zero) {
  if (slotFree_.empty()) {
    void* p = nullptr;
    bool pinned = ugo_fec_host_alloc(kSlabSlots * kSlotStride, &p) == UGO_FEC_OK;
    if (!pinned) p = std::aligned_alloc(16, kSlabSlots * kSlotStride);
    if (!p) std::abort();  // out of host memory, as Go's make would panic
    auto* base = static_cast<uint8_t*>(p);
    uint64_t dev = 0;
    if (pinned) {
      void* d = nullptr;
      if (ugo_fec_device_address(enc_->handle(), base, &d) == UGO_FEC_OK) dev = reinterpret_cast<uint64_t>(d);
    }
    slabs_.push_back(base);
    slabPinned_.push_back(pinned ? 1 : 0);
    const uint32_t first = static_cast<uint32_t>(slotPtr_.size());
    for (size_t i = 0; i < kSlabSlots; ++i) {
      slotPtr_.push_back(base + i * kSlotStride);
      slotDev_.push_back(dev ? dev + i * kSlotStride : 0);
      slotHeld_.push_back(0);
      slotOrphan_.push_back(0);
    }
    for (size_t i = kSlabSlots; i-- > 0;) slotFree_.push_back(first + static_cast<uint32_t>(i));
  }
  const uint32_t s = slotFree_.back();
  slotFree_.pop_back();
  if (zero) std::memset(slotPtr_[s], 0, maxPacketSize);  // make([]byte, maxPacketSize)
  return s;
}

PoolBuf* FEC::poolGet() {  // xmitBuf.Get(): the most recently Put buffer first
  if (!poolFree_.empty()) {
    PoolBuf* b = poolFree_.back();
    poolFree_.pop_back();
    return b;
  }
  poolAll_.push_back(std::make_unique<PoolBuf>());
  poolAll_.back()->slot = newSlot(true);
  return poolAll_.back().get();
}

void FEC::poolPut(PoolBuf* b) { poolFree_.push_back(b); }

// The bytes decode is about to overwrite (head [0, n)): if a pending batch
// still has to read this buffer's slot, the buffer moves to a fresh slot and
// takes its tail [n, maxPacketSize) along -- the bytes Go's reused buffer
// would still hold -- and the old slot is freed when that batch is done.
uint8_t* FEC::writable(PoolBuf* b, size_t n) {
  const uint32_t old = b->slot;
  if (slotHeld_[old]) {
    const uint32_t s = newSlot(false);
    std::memcpy(slotPtr_[s] + n, slotPtr_[old] + n, maxPacketSize - n);
    slotOrphan_[old] = 1;
    b->slot = s;
  }
  return slotPtr_[b->slot];
}

void FEC::releaseSlot(uint32_t s) {
  slotHeld_[s] = 0;
  if (slotOrphan_[s]) {
    slotOrphan_[s] = 0;
    slotFree_.push_back(s);
  }
}

void FEC::dropBuffer(PoolBuf* b) {
  for (size_t i = poolAll_.size(); i-- > 0;)
    if (poolAll_[i].get() == b) {
      if (slotHeld_[b->slot])
        slotOrphan_[b->slot] = 1;
      else
        slotFree_.push_back(b->slot);
      poolAll_.erase(poolAll_.begin() + static_cast<long>(i));
      return;
    }
}

fecPacket FEC::decode(const uint8_t* data, size_t len) {  // :78-89
  fecPacket pkt;
  pkt.seqid = getLE32(data);
  pkt.flag = getLE16(data + 4);
  pkt.ts = clock_();
  PoolBuf* buf = poolGet();
  const size_t n = len > fecHeaderSize ? std::min(maxPacketSize, len - fecHeaderSize) : 0;
  uint8_t* dst = writable(buf, n);
  if (n) std::memcpy(dst, data + fecHeaderSize, n);  // copy(buf, data[6:]); stale tail kept
  pkt.data = buf;
  return pkt;
}

void FEC::markData(uint8_t* data) {  // :91-95
  putLE32(data, next_);
  putLE16(data + 4, typeData);
  next_++;
}

void FEC::markFEC(uint8_t* data) {  // :97-104
  putLE32(data, next_);
  putLE16(data + 4, typeFEC);
  next_++;
  if (next_ >= paws_) next_ = 0;
}

std::vector<Bytes> FEC::input(fecPacket pkt) {  // :107-226
  std::vector<Bytes> recovered;
  lastError_ = UGO_FEC_OK;  // this call's own status (an earlier call's error is not this one's)
  const uint32_t now = clock_();
  if (now - lastCheck_ >= fecExpire) {  // expiration :109-121
    std::vector<fecPacket> keep;
    for (auto& q : rx_) {
      if (now - q.ts < fecExpire)
        keep.push_back(q);
      else
        poolPut(q.data);
    }
    rx_.swap(keep);
    lastCheck_ = now;
  }
  // insertion :124-143
  const int n = static_cast<int>(rx_.size()) - 1;
  int insertIdx = 0;
  for (int i = n; i >= 0; --i) {
    if (pkt.seqid == rx_[i].seqid) {  // de-duplicate
      poolPut(pkt.data);
      return recovered;
    } else if (pkt.seqid > rx_[i].seqid) {
      insertIdx = i + 1;
      break;
    }
  }
  rx_.insert(rx_.begin() + insertIdx, pkt);

  const uint32_t ss = uint32_t(shardSize_);
  const uint32_t shardBegin = pkt.seqid - pkt.seqid % ss;  // :145-146
  const uint32_t shardEnd = shardBegin + ss - 1;
  int searchBegin = insertIdx - shardSize_;
  if (searchBegin < 0) searchBegin = 0;
  int searchEnd = insertIdx + shardSize_;
  if (searchEnd >= static_cast<int>(rx_.size())) searchEnd = static_cast<int>(rx_.size()) - 1;

  if (static_cast<int>(rx_.size()) >= dataShards_ && shardBegin < shardEnd) {  // :158
    int numshard = 0, numDataShard = 0, first = -1;
    size_t maxlen = 0;
    std::vector<PoolBuf*> shards(shardSize_, nullptr);
    for (int i = searchBegin; i <= searchEnd; ++i) {  // :170-188
      const uint32_t seqid = rx_[i].seqid;
      if (seqid > shardEnd) break;
      if (seqid >= shardBegin) {
        shards[seqid % ss] = rx_[i].data;
        numshard++;
        if (rx_[i].flag == typeData) numDataShard++;
        if (numshard == 1) first = i;
        maxlen = maxPacketSize;  // len(rx[i].data): every pool buffer is maxPacketSize long
      }
    }
    if (numDataShard == dataShards_) {  // no loss :190-195
      for (int i = first; i < first + numshard; ++i) poolPut(rx_[i].data);
      rx_.erase(rx_.begin() + first, rx_.begin() + first + numshard);
    } else if (numshard >= dataShards_) {  // recoverable :196-217
      recoverGroup(shards, maxlen, recovered);
      for (int i = first; i < first + numshard; ++i) poolPut(rx_[i].data);
      rx_.erase(rx_.begin() + first, rx_.begin() + first + numshard);
    }
  }
  if (static_cast<int>(rx_.size()) > rxlimit_) {  // keep rxlimit :220-224
    poolPut(rx_.front().data);
    rx_.erase(rx_.begin());
  }
  return recovered;
}

// --------------------------------------------------------------- recovery

bool FEC::ensureGpu() {
  if (stream_) return true;
  DevGuard g(device_);
  if (hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking) != hipSuccess) {
    stream_ = nullptr;
    return false;
  }
  return true;
}

void FEC::freeBatch(Batch& b) {
  if (b.mem) ugo_fec_host_free(b.mem);
  if (b.done) (void)hipEventDestroy(b.done);
  b = Batch{};
}

// Pinned [rows | masks | status | out] for `cap` groups (empty batch only).
// The new memory is allocated before the old is freed: on failure the batch
// keeps what it had (setBatch then drops back to per-call recovery).
bool FEC::ensureBatch(Batch& b, size_t cap) {
  if (b.mem && b.cap >= cap) return true;
  const size_t n = static_cast<size_t>(shardSize_), slots = outSlots();
  const size_t o_rows = 0, o_masks = o_rows + cap * n * 8, o_status = o_masks + cap * 8;
  const size_t o_out = (o_status + cap + 15) / 16 * 16, bytes = o_out + cap * slots * kSlotStride;
  void* p = nullptr;
  if (ugo_fec_host_alloc(bytes, &p) != UGO_FEC_OK) return false;
  if (!b.done) {
    DevGuard g(device_);
    if (hipEventCreateWithFlags(&b.done, hipEventDisableTiming) != hipSuccess) {
      ugo_fec_host_free(p);
      b.done = nullptr;
      return false;
    }
  }
  if (b.mem) ugo_fec_host_free(b.mem);
  b.mem = static_cast<uint8_t*>(p);
  b.cap = cap;
  b.rows = reinterpret_cast<uint64_t*>(b.mem + o_rows);
  b.masks = reinterpret_cast<uint64_t*>(b.mem + o_masks);
  b.status = reinterpret_cast<int8_t*>(b.mem + o_status);
  b.out = b.mem + o_out;
  return true;
}

// Record one recoverable group: the first d present rows (the survivors
// Reconstruct uses; input keeps only data shards, :203-207, so the rows left
// out are parity rows a data-only recovery never rebuilds) by their slots'
// device addresses.  False if a survivor's slot is not GPU-visible.
bool FEC::stage(Batch& b, const std::vector<PoolBuf*>& shards, size_t maxlen) {
  const size_t n = static_cast<size_t>(shardSize_);
  uint64_t* row = b.rows + b.groups * n;
  uint64_t mask = 0;
  int kept = 0;
  for (size_t k = 0, seen = 0; k < n && seen < static_cast<size_t>(dataShards_); ++k)
    if (shards[k]) {
      if (!slotDev_[shards[k]->slot]) return false;
      ++seen;
    }
  for (size_t k = 0; k < n; ++k) {
    row[k] = 0;
    if (shards[k] && kept < dataShards_) {
      const uint32_t s = shards[k]->slot;
      row[k] = slotDev_[s];  // shards[k][:maxlen], read in place
      mask |= 1ull << k;
      ++kept;
      if (!slotHeld_[s]) {
        slotHeld_[s] = 1;
        b.held.push_back(s);
      }
    }
  }
  b.masks[b.groups] = mask;
  b.S = maxlen;
  ++b.groups;
  return true;
}

bool FEC::launch(Batch& b) {
  DevGuard g(device_);
  int st = ugo_fec_reconstruct_rows(enc_->handle(), reinterpret_cast<const uint8_t* const*>(b.rows), b.masks,
                                    b.groups, b.S, b.out, kSlotStride, outSlots() * kSlotStride,
                                    UGO_FEC_RECONSTRUCT_DATA_ONLY, b.status, stream_);
  if (st == UGO_FEC_OK && hipEventRecord(b.done, stream_) != hipSuccess) st = UGO_FEC_ERR_HIP;
  lastError_ = st;
  b.err = st;
  b.inflight = true;  // collect() waits (if launched) and releases the slots either way
  return st == UGO_FEC_OK;
}

// Wait for a launched batch and append its recovered data shards, group by
// group, each group's erased data rows in index order.  A group whose status
// is not OK yields nothing, as a failing per-call Reconstruct does (:208-210).
void FEC::collect(Batch& b, std::vector<Bytes>& out) {
  if (!b.inflight) return;
  const bool ok = b.err == UGO_FEC_OK && hipEventSynchronize(b.done) == hipSuccess;
  if (!ok) lastError_ = b.err ? b.err : UGO_FEC_ERR_HIP;
  const size_t d = static_cast<size_t>(dataShards_);
  if (ok) {
    for (size_t g = 0; g < b.groups; ++g) {
      if (b.status[g] != 0) continue;
      const uint8_t* grp = b.out + g * outSlots() * kSlotStride;
      size_t i = 0;
      for (size_t k = 0; k < d; ++k)
        if (!((b.masks[g] >> k) & 1ull)) {
          out.emplace_back(grp + i * kSlotStride, grp + i * kSlotStride + b.S);
          ++i;
        }
    }
  }
  for (uint32_t s : b.held) releaseSlot(s);
  b.held.clear();
  b.groups = 0;
  b.inflight = false;
}

// The filled current batch: launched and (flags 0) collected now, or
// (kBatchOverlap) left running while the previous one is collected.
void FEC::launchCurrent(std::vector<Bytes>& out) {
  Batch& b = batch_[cur_];
  if (b.groups == 0) return;
  if (!(batchFlags_ & kBatchOverlap)) {
    launch(b);
    collect(b, out);
    return;
  }
  Batch& prev = batch_[cur_ ^ 1];
  collect(prev, out);  // older shards first
  launch(b);
  cur_ ^= 1;
}

// The recoverable branch of input (ugo/fec.go:196-217): reslice to maxlen,
// Reconstruct (:202, on the GPU), append the erased data shards in index
// order (:203-207).  Per call: recoverOne.  Batched: the group joins the
// current batch, its survivors read in place.
void FEC::recoverGroup(const std::vector<PoolBuf*>& shards, size_t maxlen, std::vector<Bytes>& out) {
  if (ensureGpu()) {
    if (batchCap_ > 0) {
      Batch& b = batch_[cur_];
      if (b.groups && maxlen != b.S) launchCurrent(out);  // one shard size per batch
      Batch& c = batch_[cur_];
      if (stage(c, shards, maxlen)) {
        if (c.groups == static_cast<size_t>(batchCap_)) launchCurrent(out);
        return;
      }
      flushInto(out);  // the copy path below returns at once: pending groups first, in order
    } else if (recoverOne(shards, maxlen, out)) {
      return;
    }
  }
  // no GPU-visible pool slot (pinned memory ran out) or no stream: this group
  // through the encoder's own staging -- the data-only form over the first d
  // present rows gives the same bytes as Reconstruct's data rows
  std::vector<Bytes> rs(shardSize_);
  int kept = 0;
  for (int k = 0; k < shardSize_ && kept < dataShards_; ++k)
    if (shards[k]) {
      const uint8_t* src = slotPtr_[shards[k]->slot];
      rs[k].assign(src, src + maxlen);  // shards[k][:maxlen]
      ++kept;
    }
  const int err = enc_->ReconstructData(rs);  // -> GPU
  lastError_ = err;
  if (err == UGO_FEC_OK) {
    for (int k = 0; k < dataShards_; ++k)
      if (!shards[k]) out.push_back(std::move(rs[k]));
  }  // else: logged and swallowed upstream (:208-210)
}

// Per call: the survivors are copied into a pinned one-group stage and
// recovered zero-copy (ugo_fec_reconstruct_host), waited for here.  For a
// single group this beats reading them in place (ugo_fec_reconstruct_rows):
// 7.3 vs 12.2 us of kernel, the extra row-pointer round trip over PCIe and the
// larger kernel outweighing the 15 KB copy (profiles/r3/rows_probe2.jsonl).
bool FEC::recoverOne(const std::vector<PoolBuf*>& shards, size_t maxlen, std::vector<Bytes>& out) {
  const size_t n = static_cast<size_t>(shardSize_);
  const size_t pitch = (maxlen + 15) / 16 * 16;
  if (!one_ || oneBytes_ < n * pitch) {
    if (one_) ugo_fec_host_free(one_);
    one_ = nullptr;
    oneBytes_ = 0;
    void* p = nullptr;
    if (ugo_fec_host_alloc(n * pitch, &p) != UGO_FEC_OK) return false;
    one_ = static_cast<uint8_t*>(p);
    oneBytes_ = n * pitch;
  }
  uint64_t mask = 0;
  int kept = 0;
  for (size_t k = 0; k < n && kept < dataShards_; ++k)
    if (shards[k]) {
      std::memcpy(one_ + k * pitch, slotPtr_[shards[k]->slot], maxlen);  // shards[k][:maxlen]
      mask |= 1ull << k;
      ++kept;
    }
  int8_t status = 0;
  const int err = ugo_fec_reconstruct_host(enc_->handle(), one_, &mask, 1, maxlen, pitch,
                                           UGO_FEC_RECONSTRUCT_DATA_ONLY, &status);  // :202 -> GPU
  lastError_ = err;
  if (err == UGO_FEC_OK)
    for (int k = 0; k < dataShards_; ++k)
      if (!shards[k]) out.emplace_back(one_ + k * pitch, one_ + k * pitch + maxlen);
  return err != UGO_FEC_ERR_HIP;  // a failing Reconstruct is logged and swallowed upstream (:208-210)
}

void FEC::flushInto(std::vector<Bytes>& out) {
  Batch& prev = batch_[cur_ ^ 1];
  collect(prev, out);  // an overlapped batch still running: older shards first
  Batch& b = batch_[cur_];
  if (b.groups) {
    launch(b);
    collect(b, out);
  }
}

std::vector<Bytes> FEC::flush() {
  std::vector<Bytes> out;
  lastError_ = UGO_FEC_OK;
  flushInto(out);
  return out;
}

size_t FEC::pending() const {
  return batch_[0].groups + batch_[1].groups;
}

size_t FEC::maxReturnGroups(bool isFlush) const {
  const size_t cap = static_cast<size_t>(batchCap_);
  if (cap == 0) return isFlush ? 0 : 1;
  // overlap: the previous batch and the current one -- flush, and input when a
  // group cannot be staged (no GPU-visible pool slot: recoverGroup flushes
  // both, then recovers that group by copy); without overlap the current
  // batch, or the current batch's cap - 1 groups plus that group
  if (batchFlags_ & kBatchOverlap) return 2 * cap;
  return cap;
}

std::vector<Bytes> FEC::setBatch(int groups, unsigned flags) {
  std::vector<Bytes> out;
  if (groups < 0 || (groups > 0 && shardSize_ > 64) || (flags & ~kBatchOverlap)) {
    lastError_ = UGO_FEC_ERR_INVALID_ARG;
    return out;
  }
  flushInto(out);
  lastError_ = UGO_FEC_OK;
  if (groups > 0) {
    if (!ensureGpu() || !ensureBatch(batch_[0], size_t(groups)) ||
        ((flags & kBatchOverlap) && !ensureBatch(batch_[1], size_t(groups)))) {
      // no room for the batch: per-call recovery (a batch smaller than asked
      // for is never used -- the pending batches are empty after flushInto)
      batchCap_ = 0;
      batchFlags_ = 0;
      cur_ = 0;
      lastError_ = UGO_FEC_ERR_HIP;
      return out;
    }
  }
  batchCap_ = groups;
  batchFlags_ = groups > 0 ? flags : 0;
  cur_ = 0;
  return out;
}

FEC::~FEC() {
  if (one_) ugo_fec_host_free(one_);
  for (Batch& b : batch_) {
    if (b.inflight && b.done) (void)hipEventSynchronize(b.done);
    freeBatch(b);
  }
  if (stream_) {
    DevGuard g(device_);
    (void)hipStreamDestroy(stream_);
  }
  for (size_t i = 0; i < slabs_.size(); ++i) {
    if (slabPinned_[i])
      ugo_fec_host_free(slabs_[i]);
    else
      std::free(slabs_[i]);
  }
}

int FEC::calcECC(uint8_t* const* bufs, const size_t* lens, int n, int offset, int maxlen) {  // :228-243
  if (n != shardSize_) return lastError_ = UGO_FEC_ERR_INVALID_ARG;  // "mismatch" logged upstream
  if (offset < 0 || maxlen < offset) return lastError_ = UGO_FEC_ERR_INVALID_ARG;  // Go: slice bounds panic
  uint8_t* rows[256];
  for (int k = 0; k < n; ++k) {
    if (lens[k] < static_cast<size_t>(maxlen)) return lastError_ = UGO_FEC_ERR_INVALID_ARG;  // slice bounds
    rows[k] = bufs[k] + offset;
  }
  return lastError_ = enc_->EncodeWindows(rows, size_t(maxlen - offset));  // :238 -> GPU
}

std::vector<Bytes*> FEC::calcECC(std::vector<Bytes>& data, int offset, int maxlen) {  // :228-243
  std::vector<Bytes*> ecc;
  std::vector<uint8_t*> bufs(data.size());
  std::vector<size_t> lens(data.size());
  for (size_t k = 0; k < data.size(); ++k) {
    bufs[k] = data[k].data();
    lens[k] = data[k].size();
  }
  if (calcECC(bufs.data(), lens.data(), static_cast<int>(data.size()), offset, maxlen) != UGO_FEC_OK) return ecc;
  for (int k = dataShards_; k < shardSize_; ++k) ecc.push_back(&data[k]);
  return ecc;
}

int FEC::service(int idle_us) {
  return idle_us < 0 ? enc_->ServiceStop() : enc_->ServiceStart(static_cast<unsigned>(idle_us));
}

}  // namespace ugo
