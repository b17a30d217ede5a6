// conn_abi.cpp -- C-ABI (include/ugo_fec_conn.h) over the C++ FEC mirror.
#include "../../../include/ugo_fec_conn.h"

#include <cstring>
#include <new>

#include "fec.hpp"

struct ugo_fecconn {
  std::unique_ptr<ugo::FEC> fec;
};

namespace {

// Recovered shards out at a UGO_FEC_MAX_PACKET stride; every shard of one
// call has the same length (the pool's buffers are all maxPacketSize long).
int emit(const std::vector<ugo::Bytes>& rec, uint8_t* out, size_t out_cap, int* nrec, size_t* rec_len) {
  if (rec.empty()) return UGO_FEC_OK;
  const size_t L = rec[0].size();
  if (!out || out_cap < rec.size() * ugo::maxPacketSize || L > ugo::maxPacketSize) return UGO_FEC_ERR_INVALID_ARG;
  for (size_t i = 0; i < rec.size(); ++i) {
    if (rec[i].size() != L) return UGO_FEC_ERR_INVALID_ARG;
    std::memcpy(out + i * ugo::maxPacketSize, rec[i].data(), L);
  }
  if (nrec) *nrec = static_cast<int>(rec.size());
  if (rec_len) *rec_len = L;
  return UGO_FEC_OK;
}

// The caller's buffer must hold the most one call can return before anything
// is consumed (a packet taken into the rx queue whose recovered shards then
// fail to fit would lose them): a whole batch of groups in batch mode, and for
// input in per-call mode one group's d shards.  set_batch / flush in per-call
// mode have nothing pending to return.
bool batch_cap_ok(const ugo_fecconn* f, const uint8_t* out, size_t out_cap, bool is_flush = false) {
  const size_t groups = f->fec->maxReturnGroups(is_flush);
  if (groups == 0) return true;
  return out && out_cap >= groups * static_cast<size_t>(f->fec->dataShards()) * ugo::maxPacketSize;
}

}  // namespace

extern "C" {

int ugo_fecconn_new(int rxlimit, int d, int p, int device, ugo_fecconn** out) {
  if (!out) return UGO_FEC_ERR_INVALID_ARG;
  *out = nullptr;
  if (d <= 0 || p <= 0 || rxlimit < d + p) return UGO_FEC_ERR_INV_SHARD_NUM;  // newFEC -> nil
  // probe reedsolomon.New's status for a precise error before constructing
  ugo_fec* probe = nullptr;
  const int st = ugo_fec_create(device, d, p, &probe);
  if (st != UGO_FEC_OK) return st;
  ugo_fec_destroy(probe);
  auto* c = new (std::nothrow) ugo_fecconn();
  if (!c) return UGO_FEC_ERR_INVALID_ARG;
  c->fec = ugo::FEC::newFEC(rxlimit, d, p, device);
  if (!c->fec) {
    delete c;
    return UGO_FEC_ERR_HIP;
  }
  *out = c;
  return UGO_FEC_OK;
}

void ugo_fecconn_free(ugo_fecconn* f) { delete f; }

int ugo_fecconn_set_clock(ugo_fecconn* f, uint32_t (*clock)(void*), void* user) {
  if (!f) return UGO_FEC_ERR_INVALID_ARG;
  if (clock)
    f->fec->setClock([clock, user]() { return clock(user); });
  else
    f->fec->setClock(ugo::currentMs);
  return UGO_FEC_OK;
}

int ugo_fecconn_mark_data(ugo_fecconn* f, uint8_t* data) {
  if (!f || !data) return UGO_FEC_ERR_INVALID_ARG;
  f->fec->markData(data);
  return UGO_FEC_OK;
}

int ugo_fecconn_mark_fec(ugo_fecconn* f, uint8_t* data) {
  if (!f || !data) return UGO_FEC_ERR_INVALID_ARG;
  f->fec->markFEC(data);
  return UGO_FEC_OK;
}

int ugo_fecconn_get_next(const ugo_fecconn* f, uint32_t* next) {
  if (!f || !next) return UGO_FEC_ERR_INVALID_ARG;
  *next = f->fec->next();
  return UGO_FEC_OK;
}

int ugo_fecconn_set_next(ugo_fecconn* f, uint32_t next) {
  if (!f) return UGO_FEC_ERR_INVALID_ARG;
  f->fec->setNext(next);
  return UGO_FEC_OK;
}

int ugo_fecconn_input(ugo_fecconn* f, const uint8_t* wire, size_t len, uint32_t* seqid, uint16_t* flag,
                      uint8_t* out, size_t out_cap, int* nrec, size_t* rec_len) {
  if (!f || !wire || len < ugo::fecHeaderSize) return UGO_FEC_ERR_INVALID_ARG;
  if (nrec) *nrec = 0;
  if (rec_len) *rec_len = 0;
  if (!batch_cap_ok(f, out, out_cap)) return UGO_FEC_ERR_INVALID_ARG;
  ugo::fecPacket pkt = f->fec->decode(wire, len);
  if (seqid) *seqid = pkt.seqid;
  if (flag) *flag = pkt.flag;
  if (pkt.flag != ugo::typeData && pkt.flag != ugo::typeFEC) {
    // ugo/conn.go:395: such a packet never reaches input(); its pool buffer
    // is dropped (never Put back), as in Go
    f->fec->dropBuffer(pkt.data);
    return UGO_FEC_OK;
  }
  std::vector<ugo::Bytes> rec = f->fec->input(pkt);
  const int st = emit(rec, out, out_cap, nrec, rec_len);
  if (st) return st;
  return f->fec->lastError() == UGO_FEC_ERR_HIP ? UGO_FEC_ERR_HIP : UGO_FEC_OK;
}

int ugo_fecconn_set_batch_ex(ugo_fecconn* f, int groups, unsigned flags, uint8_t* out, size_t out_cap, int* nrec,
                             size_t* rec_len) {
  if (nrec) *nrec = 0;
  if (rec_len) *rec_len = 0;
  if (!f || groups < 0 || (groups > 0 && f->fec->dataShards() + f->fec->parityShards() > 64) ||
      (flags & ~UGO_FECCONN_BATCH_OVERLAP))
    return UGO_FEC_ERR_INVALID_ARG;
  if (!batch_cap_ok(f, out, out_cap, true)) return UGO_FEC_ERR_INVALID_ARG;  // what is pending comes back
  std::vector<ugo::Bytes> rec = f->fec->setBatch(groups, flags);
  const int st = emit(rec, out, out_cap, nrec, rec_len);
  if (st) return st;
  return f->fec->lastError() == UGO_FEC_ERR_HIP ? UGO_FEC_ERR_HIP : UGO_FEC_OK;
}

int ugo_fecconn_set_batch(ugo_fecconn* f, int groups, uint8_t* out, size_t out_cap, int* nrec, size_t* rec_len) {
  return ugo_fecconn_set_batch_ex(f, groups, 0, out, out_cap, nrec, rec_len);
}

int ugo_fecconn_flush(ugo_fecconn* f, uint8_t* out, size_t out_cap, int* nrec, size_t* rec_len) {
  if (nrec) *nrec = 0;
  if (rec_len) *rec_len = 0;
  if (!f || !batch_cap_ok(f, out, out_cap, true)) return UGO_FEC_ERR_INVALID_ARG;
  std::vector<ugo::Bytes> rec = f->fec->flush();
  const int st = emit(rec, out, out_cap, nrec, rec_len);
  if (st) return st;
  return f->fec->lastError() == UGO_FEC_ERR_HIP ? UGO_FEC_ERR_HIP : UGO_FEC_OK;
}

int ugo_fecconn_service(ugo_fecconn* f, int idle_us) {
  if (!f) return UGO_FEC_ERR_INVALID_ARG;
  return f->fec->service(idle_us);
}

int ugo_fecconn_pending(const ugo_fecconn* f, size_t* groups) {
  if (!f || !groups) return UGO_FEC_ERR_INVALID_ARG;
  *groups = f->fec->pending();
  return UGO_FEC_OK;
}

int ugo_fecconn_calc_ecc(ugo_fecconn* f, uint8_t* const* bufs, const size_t* lens, int n, int offset, int maxlen) {
  if (!f || !bufs || !lens || n < 0) return UGO_FEC_ERR_INVALID_ARG;
  return f->fec->calcECC(bufs, lens, n, offset, maxlen);  // in place on the caller's packets
}

int ugo_fecconn_rx_len(const ugo_fecconn* f, size_t* len) {
  if (!f || !len) return UGO_FEC_ERR_INVALID_ARG;
  *len = f->fec->rxLen();
  return UGO_FEC_OK;
}

}  // extern "C"
