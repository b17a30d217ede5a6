// reedsolomon.hpp -- C++ host mirror of the klauspost/reedsolomon Encoder
// subset that jflyup/ugo uses (New ugo/fec.go:59, Reconstruct :202,
// Encode :238), over the MI355X C-ABI (include/ugo_fec.h).
//
// Go's [][]byte becomes std::vector<Bytes>; a nil / empty shard is an empty
// Bytes (len 0), exactly the "len(shards[i]) != 0" presence test upstream.
// Errors are returned as ugo_fec_status codes (0 = nil error).
#pragma once
#include <cstddef>
#include <cstdint>
#include <memory>
#include <vector>

#include "../../../include/ugo_fec.h"

namespace ugo {

using Bytes = std::vector<uint8_t>;

namespace reedsolomon {

class Encoder {
 public:
  Encoder(const Encoder&) = delete;
  Encoder& operator=(const Encoder&) = delete;
  ~Encoder();

  // Encode: parity shards [d, d+p) written in place from data shards [0, d).
  int Encode(std::vector<Bytes>& shards);
  // Encode over raw windows (calcECC's data[k][offset:maxlen], ugo/fec.go:235).
  int EncodeWindows(uint8_t* const* rows, size_t shard_size);
  // Reconstruct: every empty shard is rebuilt (data and parity).
  int Reconstruct(std::vector<Bytes>& shards);
  int ReconstructData(std::vector<Bytes>& shards);
  // Reconstruct every group of a pinned group-major batch [G][d+p][pitch]
  // (ugo_fec_reconstruct_host): the batched form of G Reconstruct calls,
  // one launch.  status (G entries, nullable) gets each group's status.
  int ReconstructBatch(uint8_t* batch, const uint64_t* present, size_t groups, size_t shard_size,
                       size_t pitch, unsigned flags, int8_t* status);

  // Per-call latency service (ugo_fec_service_start): the one-group Encode /
  // Reconstruct calls above are served by a resident workgroup, no launch
  // each (the cgo shim's ServiceStart).
  int ServiceStart(unsigned idle_us = 0) { return ugo_fec_service_start(ctx_, idle_us); }
  int ServiceStop() { return ugo_fec_service_stop(ctx_); }

  int DataShards() const { return d_; }
  int ParityShards() const { return p_; }
  int Shards() const { return d_ + p_; }
  ugo_fec* handle() const { return ctx_; }

 private:
  friend std::unique_ptr<Encoder> New(int, int, int*, int);
  Encoder(ugo_fec* ctx, int d, int p) : ctx_(ctx), d_(d), p_(p) {}
  uint8_t* staging(size_t bytes);
  int reconstruct(std::vector<Bytes>& shards, unsigned flags);

  ugo_fec* ctx_;
  int d_, p_;
  uint8_t* stage_ = nullptr;  // pinned host staging, one group [d+p][S]
  size_t stage_bytes_ = 0;
};

// reedsolomon.New(dataShards, parityShards); *err receives the status.
std::unique_ptr<Encoder> New(int dataShards, int parityShards, int* err, int device = 0);

}  // namespace reedsolomon
}  // namespace ugo
