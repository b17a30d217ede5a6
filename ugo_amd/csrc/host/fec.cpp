// fec.cpp -- see fec.hpp.  Control logic mirrors ugo/fec.go line by line in
// behaviour; every byte of Reed-Solomon arithmetic runs on the GPU through
// reedsolomon::Encoder (the C-ABI), none on the CPU.
#include "fec.hpp"

#include <chrono>
#include <cstring>

namespace ugo {

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
  f->paws_ = (0xffffffffu / uint32_t(f->shardSize_) - 1) * uint32_t(f->shardSize_);  // :58
  int err = 0;
  f->enc_ = reedsolomon::New(dataShards, parityShards, &err, device);  // :59
  if (!f->enc_) return nullptr;  // :60-63 (logged upstream)
  f->clock_ = currentMs;
  return f;
}

Bytes* FEC::poolGet() {
  if (!poolFree_.empty()) {
    Bytes* b = poolFree_.back();
    poolFree_.pop_back();
    return b;
  }
  poolAll_.push_back(std::make_unique<Bytes>(maxPacketSize, 0));
  return poolAll_.back().get();
}

void FEC::poolPut(Bytes* b) { poolFree_.push_back(b); }

void FEC::dropBuffer(Bytes* b) {
  for (size_t i = poolAll_.size(); i-- > 0;)
    if (poolAll_[i].get() == b) {
      poolAll_.erase(poolAll_.begin() + static_cast<long>(i));
      return;
    }
}

fecPacket FEC::decode(const uint8_t* data, size_t len) {  // :78-89
  fecPacket pkt;
  pkt.seqid = getLE32(data);
  pkt.flag = getLE16(data + 4);
  pkt.ts = clock_();
  Bytes* buf = poolGet();
  const size_t n = len > fecHeaderSize ? std::min(buf->size(), len - fecHeaderSize) : 0;
  if (n) std::memcpy(buf->data(), data + fecHeaderSize, n);  // copy(buf, data[6:]); stale tail kept
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
    std::vector<Bytes*> shards(shardSize_, nullptr);
    for (int i = searchBegin; i <= searchEnd; ++i) {  // :170-188
      const uint32_t seqid = rx_[i].seqid;
      if (seqid > shardEnd) break;
      if (seqid >= shardBegin) {
        shards[seqid % ss] = rx_[i].data;
        numshard++;
        if (rx_[i].flag == typeData) numDataShard++;
        if (numshard == 1) first = i;
        if (rx_[i].data->size() > maxlen) maxlen = rx_[i].data->size();
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

// The recoverable branch of input (ugo/fec.go:196-217).  Per call: reslice
// to maxlen, Reconstruct (:202, on the GPU), append the erased data shards in
// index order (:203-207).  Batched: the same bytes are staged and recovered
// with the rest of the batch (flushInto), so the result is identical.
void FEC::recoverGroup(const std::vector<Bytes*>& shards, size_t maxlen, std::vector<Bytes>& out) {
  if (batchCap_ > 0) {
    const size_t n = static_cast<size_t>(shardSize_);
    const size_t pitch = (maxlen + 15) / 16 * 16;
    if (!pendMask_.empty() && maxlen != batchS_) flushInto(out);  // one shard size per batch
    const size_t need = static_cast<size_t>(batchCap_) * n * pitch;
    if (need > batchBytes_) {  // pendMask_ is empty here
      if (batchBuf_) ugo_fec_host_free(batchBuf_);
      batchBuf_ = nullptr;
      batchBytes_ = 0;
      void* p = nullptr;
      if (ugo_fec_host_alloc(need, &p) == UGO_FEC_OK) {
        batchBuf_ = static_cast<uint8_t*>(p);
        batchBytes_ = need;
      }
    }
    if (batchBuf_) {
      batchS_ = maxlen;
      batchPitch_ = pitch;
      uint8_t* grp = batchBuf_ + pendMask_.size() * n * pitch;
      // Only the survivors Reconstruct uses -- the first d present rows -- are
      // staged: the present data rows all come first, so the rows left out are
      // parity rows, which a data-only recovery never rebuilds.  Same result,
      // fewer bytes copied.
      uint64_t mask = 0;
      int kept = 0;
      for (size_t k = 0; k < n && kept < dataShards_; ++k)
        if (shards[k]) {
          std::memcpy(grp + k * pitch, shards[k]->data(), maxlen);  // shards[k][:maxlen]
          mask |= 1ull << k;
          ++kept;
        }
      pendMask_.push_back(mask);
      if (pendMask_.size() == static_cast<size_t>(batchCap_)) flushInto(out);
      return;
    }
    lastError_ = UGO_FEC_ERR_HIP;  // no pinned batch: recover this group per call
  }
  // :202 Reconstruct, of which input keeps the data shards (:203-207): the
  // data-only form over the first d present rows gives those same bytes
  std::vector<Bytes> rs(shardSize_);
  int kept = 0;
  for (int k = 0; k < shardSize_ && kept < dataShards_; ++k)
    if (shards[k]) {
      rs[k].assign(shards[k]->begin(), shards[k]->begin() + maxlen);  // shards[k][:maxlen]
      ++kept;
    }
  const int err = enc_->ReconstructData(rs);  // -> GPU
  lastError_ = err;
  if (err == UGO_FEC_OK) {
    for (int k = 0; k < dataShards_; ++k)
      if (!shards[k]) out.push_back(std::move(rs[k]));
  }  // else: logged and swallowed upstream (:208-210)
}

// One launch over the pending groups (data rows only: input returns data
// shards, :203-207).  A group whose status is not OK yields nothing, as a
// failing per-call Reconstruct does.
void FEC::flushInto(std::vector<Bytes>& out) {
  const size_t G = pendMask_.size();
  if (G == 0) return;
  const size_t n = static_cast<size_t>(shardSize_);
  std::vector<int8_t> st(G, 0);
  const int err = enc_->ReconstructBatch(batchBuf_, pendMask_.data(), G, batchS_, batchPitch_,
                                         UGO_FEC_RECONSTRUCT_DATA_ONLY, st.data());
  lastError_ = err;
  if (err != UGO_FEC_ERR_HIP) {
    for (size_t g = 0; g < G; ++g) {
      if (st[g] != 0) continue;
      const uint8_t* grp = batchBuf_ + g * n * batchPitch_;
      for (int k = 0; k < dataShards_; ++k)
        if (!((pendMask_[g] >> k) & 1ull)) out.emplace_back(grp + k * batchPitch_, grp + k * batchPitch_ + batchS_);
    }
  }
  pendMask_.clear();
}

std::vector<Bytes> FEC::flush() {
  std::vector<Bytes> out;
  flushInto(out);
  return out;
}

std::vector<Bytes> FEC::setBatch(int groups) {
  std::vector<Bytes> out;
  if (groups < 0 || (groups > 0 && shardSize_ > 64)) {
    lastError_ = UGO_FEC_ERR_INVALID_ARG;
    return out;
  }
  flushInto(out);
  batchCap_ = groups;
  lastError_ = UGO_FEC_OK;
  return out;
}

FEC::~FEC() {
  if (batchBuf_) ugo_fec_host_free(batchBuf_);
}

std::vector<Bytes*> FEC::calcECC(std::vector<Bytes>& data, int offset, int maxlen) {  // :228-243
  std::vector<Bytes*> ecc;
  if (static_cast<int>(data.size()) != shardSize_) {
    lastError_ = UGO_FEC_ERR_INVALID_ARG;  // "mismatch" logged upstream
    return ecc;
  }
  if (offset < 0 || maxlen < offset) {  // Go: slice bounds panic
    lastError_ = UGO_FEC_ERR_INVALID_ARG;
    return ecc;
  }
  std::vector<uint8_t*> rows(shardSize_);
  for (int k = 0; k < shardSize_; ++k) {
    if (static_cast<int>(data[k].size()) < maxlen) {  // Go: slice bounds panic
      lastError_ = UGO_FEC_ERR_INVALID_ARG;
      return ecc;
    }
    rows[k] = data[k].data() + offset;
  }
  const int err = enc_->EncodeWindows(rows.data(), size_t(maxlen - offset));  // :238 -> GPU
  lastError_ = err;
  if (err != UGO_FEC_OK) return ecc;
  for (int k = dataShards_; k < shardSize_; ++k) ecc.push_back(&data[k]);
  return ecc;
}

}  // namespace ugo
