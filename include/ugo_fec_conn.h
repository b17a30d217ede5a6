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
 * bytes available); *nrec receives their count and *rec_len their length. */
int ugo_fecconn_input(ugo_fecconn* f, const uint8_t* wire, size_t len, uint32_t* seqid, uint16_t* flag,
                      uint8_t* out, size_t out_cap, int* nrec, size_t* rec_len);

/* calcECC(data, offset, maxlen) (ugo/fec.go:228-243) over n caller buffers of
 * lengths lens[]: parity written into bufs[d..n)[offset:maxlen). */
int ugo_fecconn_calc_ecc(ugo_fecconn* f, uint8_t* const* bufs, const size_t* lens, int n, int offset,
                         int maxlen);

/* len(fec.rx): packets held in the ordered receive queue. */
int ugo_fecconn_rx_len(const ugo_fecconn* f, size_t* len);

#ifdef __cplusplus
}
#endif
#endif /* UGO_FEC_CONN_H */
