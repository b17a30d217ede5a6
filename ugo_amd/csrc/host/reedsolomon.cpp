// reedsolomon.cpp -- see reedsolomon.hpp.  One group per call, staged through
// a pinned buffer into the host-batch entry points of the C-ABI (groups = 1).
// Rows are staged at a 16-byte pitch, so the vector kernels run whatever the
// shard size (ugo's 1470-B calcECC window and 1476-B input shards are not
// multiples of 16), and the pinned stage is used zero-copy by the engine.
#include "reedsolomon.hpp"

#include <cstring>

namespace ugo {
namespace reedsolomon {

std::unique_ptr<Encoder> New(int dataShards, int parityShards, int* err, int device) {
  ugo_fec* ctx = nullptr;
  const int st = ugo_fec_create(device, dataShards, parityShards, &ctx);
  if (err) *err = st;
  if (st != UGO_FEC_OK) return nullptr;
  return std::unique_ptr<Encoder>(new Encoder(ctx, dataShards, parityShards));
}

Encoder::~Encoder() {
  if (stage_) ugo_fec_host_free(stage_);
  ugo_fec_destroy(ctx_);
}

uint8_t* Encoder::staging(size_t bytes) {
  if (bytes > stage_bytes_) {
    if (stage_) ugo_fec_host_free(stage_);
    stage_ = nullptr;
    stage_bytes_ = 0;
    void* p = nullptr;
    if (ugo_fec_host_alloc(bytes, &p) != UGO_FEC_OK) return nullptr;
    stage_ = static_cast<uint8_t*>(p);
    stage_bytes_ = bytes;
  }
  return stage_;
}

int Encoder::Encode(std::vector<Bytes>& shards) {
  const int n = Shards();
  if (static_cast<int>(shards.size()) != n) return UGO_FEC_ERR_TOO_FEW_SHARDS;
  std::vector<size_t> lens(n);
  for (int i = 0; i < n; ++i) lens[i] = shards[i].size();
  size_t S = 0;
  int st = ugo_fec_check_shards(n, lens.data(), 0, &S);
  if (st) return st;
  std::vector<uint8_t*> rows(n);
  for (int i = 0; i < n; ++i) rows[i] = shards[i].data();
  return EncodeWindows(rows.data(), S);
}

static inline size_t pitch_of(size_t S) { return (S + 15) / 16 * 16; }

int Encoder::EncodeWindows(uint8_t* const* rows, size_t S) {
  const int n = Shards();
  if (S == 0) return UGO_FEC_ERR_SHARD_NO_DATA;
  const size_t pitch = pitch_of(S);
  uint8_t* buf = staging(size_t(n) * pitch);
  if (!buf) return UGO_FEC_ERR_HIP;
  for (int k = 0; k < d_; ++k) std::memcpy(buf + size_t(k) * pitch, rows[k], S);
  const int st = ugo_fec_encode_host(ctx_, buf, 1, S, pitch);
  if (st) return st;
  for (int k = d_; k < n; ++k) std::memcpy(rows[k], buf + size_t(k) * pitch, S);
  return UGO_FEC_OK;
}

int Encoder::reconstruct(std::vector<Bytes>& shards, unsigned flags) {
  const int n = Shards();
  if (static_cast<int>(shards.size()) != n) return UGO_FEC_ERR_TOO_FEW_SHARDS;
  std::vector<size_t> lens(n);
  for (int i = 0; i < n; ++i) lens[i] = shards[i].size();
  size_t S = 0;
  int st = ugo_fec_check_shards(n, lens.data(), 1, &S);
  if (st) return st;
  const size_t pitch = pitch_of(S);
  uint8_t* buf = staging(size_t(n) * pitch);
  if (!buf) return UGO_FEC_ERR_HIP;
  uint64_t mask[4] = {0, 0, 0, 0};  // ceil(n / 64) words, n <= 256
  for (int r = 0; r < n; ++r)
    if (lens[r]) {
      mask[r >> 6] |= 1ull << (r & 63);
      std::memcpy(buf + size_t(r) * pitch, shards[r].data(), S);
    }
  int8_t status = 0;
  st = ugo_fec_reconstruct_host(ctx_, buf, mask, 1, S, pitch, flags, &status);
  if (st) return st;
  const int limit = (flags & UGO_FEC_RECONSTRUCT_DATA_ONLY) ? d_ : n;
  for (int r = 0; r < limit; ++r)
    if (!lens[r]) shards[r].assign(buf + size_t(r) * pitch, buf + size_t(r) * pitch + S);
  return UGO_FEC_OK;
}

int Encoder::ReconstructBatch(uint8_t* batch, const uint64_t* present, size_t groups, size_t S, size_t pitch,
                              unsigned flags, int8_t* status) {
  return ugo_fec_reconstruct_host(ctx_, batch, present, groups, S, pitch, flags, status);
}

int Encoder::Reconstruct(std::vector<Bytes>& shards) { return reconstruct(shards, 0); }
int Encoder::ReconstructData(std::vector<Bytes>& shards) {
  return reconstruct(shards, UGO_FEC_RECONSTRUCT_DATA_ONLY);
}

}  // namespace reedsolomon
}  // namespace ugo
