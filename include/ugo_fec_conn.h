/*
 * ugo_fec_conn.h -- C-ABI of the per-connection FEC object: the C++ host
 * mirror (ugo_amd/csrc/host/fec.cpp) of jflyup/ugo's `FEC` struct
 * (ugo/fec.go:14-27) and its methods, the direct callers of Encode and
 * Reconstruct.  Every Reed-Solomon byte is computed by the gfx950 kernels
 * behind include/ugo_fec.h.
 *
 * Status codes are ugo_fec_status (include/ugo_fec.h).  Single-owner, like
 * ugo's FEC (used only from Conn.run, ugo/conn.go:106-127).
 */
#ifndef UGO_FEC_CONN_H
#define UGO_FEC_CONN_H

#include <stddef.h>
#include <stdint.h>

#include "ugo_fec.h"

#ifdef __cplusplus
extern "C" {
#endif

#define UGO_FEC_HEADER_SIZE 6     /* fecHeaderSize, ugo/constants.go:17 */
#define UGO_FEC_TYPE_DATA 0xf1    /* typeData, ugo/constants.go:18      */
#define UGO_FEC_TYPE_FEC 0xf2     /* typeFEC,  ugo/constants.go:19      */
#define UGO_FEC_MAX_PACKET 1476   /* maxPacketSize, ugo/constants.go:29 */

typedef struct ugo_fecconn ugo_fecconn;

/* newFEC(rxlimit, d, p) (ugo/fec.go:45-72).  Returns UGO_FEC_ERR_INV_SHARD_NUM
 * where newFEC returns nil for its own geometry checks (d <= 0, p <= 0,
 * rxlimit < d+p), or the reedsolomon.New status. */
int ugo_fecconn_new(int rxlimit, int data_shards, int parity_shards, int device, ugo_fecconn** out);
void ugo_fecconn_free(ugo_fecconn* f);

/* currentMs (ugo/fec.go:73-75) replacement for tests; NULL restores the wall clock. */
int ugo_fecconn_set_clock(ugo_fecconn* f, uint32_t (*clock)(void* user), void* user);

/* markData / markFEC (ugo/fec.go:91-104): write the 6-byte header into data[0:6]. */
int ugo_fecconn_mark_data(ugo_fecconn* f, uint8_t* data);
int ugo_fecconn_mark_fec(ugo_fecconn* f, uint8_t* data);
int ugo_fecconn_get_next(const ugo_fecconn* f, uint32_t* next);
int ugo_fecconn_set_next(ugo_fecconn* f, uint32_t next);

/* The RX hook of Conn.handlePacket (ugo/conn.go:394-396): decode(wire) then,
 * when the flag is typeData or typeFEC, input(pkt).  Recovered data shards
 * (ugo/fec.go:203-207) are written to out + i*UGO_FEC_MAX_PACKET (out_cap
 * bytes available); *nrec receives their count and *rec_len their length.
 * out_cap >= d * UGO_FEC_MAX_PACKET (one group's data shards; batch mode:
 * below), checked before the packet is consumed: UGO_FEC_ERR_INVALID_ARG and
 * no state change otherwise. */
int ugo_fecconn_input(ugo_fecconn* f, const uint8_t* wire, size_t len, uint32_t* seqid, uint16_t* flag,
                      uint8_t* out, size_t out_cap, int* nrec, size_t* rec_len);

/* calcECC(data, offset, maxlen) (ugo/fec.go:228-243) over n caller buffers of
 * lengths lens[]: parity written into bufs[d..n)[offset:maxlen). */
int ugo_fecconn_calc_ecc(ugo_fecconn* f, uint8_t* const* bufs, const size_t* lens, int n, int offset,
                         int maxlen);

/* Batched recovery (a GPU extension; ugo has none).  The pool buffers decode
 * fills live in pinned host memory, and a lost group's survivors are read by
 * the GPU where they are (ugo_fec_reconstruct_rows), never copied into a
 * batch.  With groups > 0, input does not Reconstruct each recoverable lossy
 * group (ugo/fec.go:196-217) on its own: the group is recorded, and the batch
 * is recovered in ONE launch when it holds `groups` groups, or on
 * ugo_fecconn_flush.  The recovered data shards come back group by group in
 * completion order, each group's in index order -- the concatenation of what
 * per-call input returns, delayed.  The rx queue, buffer pool (LIFO order and
 * bytes, stale tails included), dedupe, expiry and rxlimit trim are unchanged.
 *   flags 0: a full batch is recovered inside the ugo_fecconn_input call that
 *     fills it, and its shards come back from that call;
 *   UGO_FECCONN_BATCH_OVERLAP: that launch runs on while input goes on with
 *     the next batch, and its shards come back from the input call that fills
 *     the NEXT batch (or from ugo_fecconn_flush): one batch later, the GPU time
 *     off the packet path.
 * Output capacity (checked before anything is consumed): ugo_fecconn_input,
 * ugo_fecconn_flush and ugo_fecconn_set_batch[_ex] need out_cap >= groups * d
 * * UGO_FEC_MAX_PACKET for the current mode's batch (per-call mode: input
 * d packets, flush nothing), and twice that with OVERLAP (the previous and the
 * current batch: flush, or an input whose group finds no GPU-visible pool
 * buffer when pinned memory has run out).  groups = 0 restores per-call
 * recovery (the default).  Both calls first flush what is pending into out.
 * UGO_FEC_ERR_INVALID_ARG for groups < 0, unknown flags or d+p > 64. */
#define UGO_FECCONN_BATCH_OVERLAP 1u
int ugo_fecconn_set_batch(ugo_fecconn* f, int groups, uint8_t* out, size_t out_cap, int* nrec,
                          size_t* rec_len);
int ugo_fecconn_set_batch_ex(ugo_fecconn* f, int groups, unsigned flags, uint8_t* out, size_t out_cap, int* nrec,
                             size_t* rec_len);
int ugo_fecconn_flush(ugo_fecconn* f, uint8_t* out, size_t out_cap, int* nrec, size_t* rec_len);
/* Lossy groups staged and not yet recovered. */
int ugo_fecconn_pending(const ugo_fecconn* f, size_t* groups);

/* Per-call latency service on this object's encoder (ugo_fec_service_start,
 * include/ugo_fec.h): calcECC's Encode and per-call recovery's Reconstruct are
 * served by a resident workgroup instead of one launch + synchronize each.
 * idle_us: how long it waits for the next call before leaving (0 = 2000);
 * idle_us < 0 stops it (ugo_fecconn_free does too). */
int ugo_fecconn_service(ugo_fecconn* f, int idle_us);

/* len(fec.rx): packets held in the ordered receive queue. */
int ugo_fecconn_rx_len(const ugo_fecconn* f, size_t* len);

#ifdef __cplusplus
}
#endif
#endif /* UGO_FEC_CONN_H */
