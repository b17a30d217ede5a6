/*
 * ugo_fec.h -- C-ABI of the MI355X-native Reed-Solomon FEC engine for
 * jflyup/ugo's per-packet-group FEC (ugo/fec.go).
 *
 * The boundary is the klauspost/reedsolomon Encoder subset that ugo/fec.go
 * actually uses (New at ugo/fec.go:59, Reconstruct at :202, Encode at :238),
 * lifted from one group per call to a batch of independent groups so one
 * gfx950 kernel launch covers thousands of packet groups.  Plain pointers and
 * sizes only; no exceptions cross the ABI; every entry point returns a
 * ugo_fec_status.
 *
 * Batch layout (device or host memory, caller-owned):
 *     shards[g][r][pitch]   g in [0, groups), r in [0, d+p)
 *   Row r < d is data shard r, row d+i is parity shard i, exactly the index
 *   order of the [][]byte passed to Encode/Reconstruct.  Bytes [0, shard_size)
 *   of a row are the shard; bytes [shard_size, pitch) are padding the engine
 *   never reads into a result and never writes.
 *   Fast path: shards 16-byte aligned and pitch % 16 == 0 (any shard_size).
 *   Any other layout is accepted and runs a slower byte-granular kernel.
 *
 * Erasures: present[g] bit r == 1  <=>  len(shards[r]) != 0 in Go terms.
 *   One uint64 per group for d+p <= 64.  Wider codes (up to upstream's 256
 *   shards) take W = ceil((d+p)/64) words per group, present[g*W + r/64] bit
 *   r%64 for shard r; their decode descriptors are built on the host per
 *   erasure pattern (cached), so a device-resident mask batch is first copied
 *   to the host (that call synchronises its stream).  RX assembly stays at
 *   d+p <= 64 (ugo uses (10,3)).
 *
 * Threading: a context is single-owner (like ugo's FEC, used only from the
 * Conn.run goroutine, ugo/conn.go:106-127).  Distinct contexts -- e.g. one per
 * GPU -- may be driven concurrently from different threads.
 *
 * Not thread-safe per context; all device work is enqueued on `stream`
 * (hipStream_t passed as void*, NULL = the legacy default stream).
 */
#ifndef UGO_FEC_H
#define UGO_FEC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: ugo_fec_rx_assemble keeps the first copy of a repeated seqid and its
 *    stats grew a fifth counter (duplicates). */
/* 3: reconstruct entry points accept d+p > 64 with ceil((d+p)/64) presence
 *    words per group (one word, as before, for d+p <= 64). */
/* 4: ugo_fec_rx_assemble keeps the first copy of a seqid across calls into one
 *    batch too (a (group, row) already present at call entry is not written). */
/* 5: ugo_fec_reconstruct_rows (row-pointer batches) and ugo_fec_device_address. */
/* 6: the per-call service (ugo_fec_service_start / _stop). */
/* 7: ugo_fec_service_config, ugo_fec_poisoned; rx_assemble places packets in
 *    destination order (index + gather) -- same results. */
/* 8: rx_assemble writes each placed row in whole 16-B chunks: its bytes
 *    [shard_size, round_up(shard_size, 16)) become zero; ugo_fec_lossy_groups,
 *    ugo_fec_reconstruct_list, ugo_fec_recover_data, ugo_fec_rx_recover_host,
 *    ugo_fec_tx_assemble_host. */
/* 9: ugo_fec_rx_assemble_frames (frame rows: each placed row holds its
 *    decrypted packet, payload at column 6); the low-priority host copy queue is
 *    on by default, and the service pool holds at most 3 queues (8 hardware
 *    queues per process, see ugo_fec_set_host_copy_queue). */
#define UGO_FEC_ABI_VERSION 9

/* Status codes.  1..5 map 1:1 onto the klauspost/reedsolomon error values
 * that ugo/fec.go logs and swallows (ugo/fec.go:60-63, 208-210, 239-241). */
typedef enum ugo_fec_status {
  UGO_FEC_OK = 0,
  UGO_FEC_ERR_INV_SHARD_NUM = 1,  /* reedsolomon.ErrInvShardNum: d <= 0 or p < 0    */
  UGO_FEC_ERR_MAX_SHARD_NUM = 2,  /* reedsolomon.ErrMaxShardNum: d + p > 256         */
  UGO_FEC_ERR_TOO_FEW_SHARDS = 3, /* reedsolomon.ErrTooFewShards                     */
  UGO_FEC_ERR_SHARD_NO_DATA = 4,  /* reedsolomon.ErrShardNoData                      */
  UGO_FEC_ERR_SHARD_SIZE = 5,     /* reedsolomon.ErrShardSize                        */
  UGO_FEC_ERR_INVALID_ARG = 6,    /* NULL pointer, pitch < shard_size, RX with d+p > 64 ... */
  UGO_FEC_ERR_SINGULAR = 7,       /* errSingular (cannot occur for this MDS code)    */
  UGO_FEC_ERR_HIP = 8,            /* HIP runtime failure (alloc, copy, launch)       */
  UGO_FEC_ERR_NO_DEVICE = 9       /* no usable gfx950 device / bad device ordinal    */
} ugo_fec_status;

/* Flags for ugo_fec_reconstruct*.  Default (0) = Reconstruct: every erased row,
 * data AND parity, is rebuilt (ugo/fec.go:202).  DATA_ONLY = ReconstructData. */
#define UGO_FEC_RECONSTRUCT_DATA_ONLY 1u

typedef struct ugo_fec ugo_fec; /* opaque: one (d,p) code bound to one device */

/* reedsolomon.New(d, p) as called at ugo/fec.go:59 (and validated by newFEC,
 * ugo/fec.go:45-64).  Binds the code to HIP device `device`, builds the
 * systematic Vandermonde-derived (d+p) x d matrix, uploads it, and (d+p <= 16)
 * precomputes the decode descriptor of every erasure pattern. */
int ugo_fec_create(int device, int data_shards, int parity_shards, ugo_fec** out);
void ugo_fec_destroy(ugo_fec* ctx);

/* Geometry and the (d+p) x d encoding matrix, row-major (test/inspection). */
int ugo_fec_geometry(const ugo_fec* ctx, int* data_shards, int* parity_shards, int* device);
int ugo_fec_matrix(const ugo_fec* ctx, uint8_t* out /* (d+p)*d bytes */);

/* ---- device-resident batch (asynchronous on `stream`) -------------------
 * Encoder.Encode(shards) (ugo/fec.go:238) for every group: reads rows [0,d),
 * writes parity rows [d, d+p) in place.  shard_size == 0 -> ERR_SHARD_NO_DATA
 * (checkShards).  `shards` is a device pointer. */
int ugo_fec_encode(ugo_fec* ctx, uint8_t* shards, size_t groups, size_t shard_size,
                   size_t pitch, void* stream);

/* Strided form of ugo_fec_encode: row r of group g is at
 *     shards + g * group_stride + r * row_stride.
 * ugo_fec_encode(pitch) == strided(row_stride = pitch, group_stride = (d+p)*pitch).
 * The shard-major ("planar") batch layout [d+p][groups][pitch] -- row_stride =
 * groups*pitch, group_stride = pitch -- turns every shard index into one
 * sequential HBM stream and is the fastest layout on MI355X.
 * No two shard slots may overlap: the smaller stride must be >= shard_size and
 * the larger one must clear a whole run of the smaller ((count - 1) * smaller
 * + shard_size), else UGO_FEC_ERR_INVALID_ARG before any launch (the same rule
 * holds for every strided batch below).
 * Fast path: shards, row_stride and group_stride all multiples of 16.
 * Dense planar rows (group_stride == shard_size, no padding; shards and
 * row_stride multiples of 16) take the vector kernels too: encode folds
 * 16/gcd(shard_size, 16) groups into one 16-B-whole pseudo-group; reconstruct
 * (d <= 16, p <= 4, shard_size >= 1009) runs on the rows' aligned chunks.
 * Padded 16-B pitches stay the faster reconstruct layout (DESIGN_HISTORY.md §3.4). */
int ugo_fec_encode_strided(ugo_fec* ctx, uint8_t* shards, size_t groups, size_t shard_size,
                           size_t row_stride, size_t group_stride, void* stream);

/* Encoder.Reconstruct(shards) (ugo/fec.go:202) for every group.  `present`
 * (device, one u64 per group; W words for d+p > 64) marks the non-empty shards.  Survivors are the first
 * d present rows in index order (upstream rule), every erased row is written.
 * Groups with fewer than d present shards are left untouched and get
 * status UGO_FEC_ERR_TOO_FEW_SHARDS; all others UGO_FEC_OK.  `status`
 * (device, int8 per group) may be NULL.  Returns launch status only. */
int ugo_fec_reconstruct(ugo_fec* ctx, uint8_t* shards, const uint64_t* present, size_t groups,
                        size_t shard_size, size_t pitch, unsigned flags, int8_t* status,
                        void* stream);

/* Strided form of ugo_fec_reconstruct (layout as ugo_fec_encode_strided). */
int ugo_fec_reconstruct_strided(ugo_fec* ctx, uint8_t* shards, const uint64_t* present, size_t groups,
                                size_t shard_size, size_t row_stride, size_t group_stride,
                                unsigned flags, int8_t* status, void* stream);

/* Reconstruct into a separate output batch (replaces the same
 * reedsolomon.Encoder.Reconstruct, ugo/fec.go:202, in the form ugo calls it:
 * erased shards are nil, ugo/fec.go:166-176, and klauspost hands them fresh
 * buffers).  `shards` is only read.  Output i of group g -- the i-th erased row
 * in ascending row order, i.e. erased data rows first, then erased parity rows
 * (DATA_ONLY: the data rows only) -- is written, shard_size bytes, to
 *     out + g*out_group_stride + i*out_row_stride,   i < p.
 * Output slots past a group's erasure count, and every slot of a group that
 * fails (status as ugo_fec_reconstruct), are left untouched.  The rows the
 * recovered data lands in are the ones ugo appends to `recovered`
 * (ugo/fec.go:203-207).  Fast path: out 16-B aligned, strides % 16 == 0. */
int ugo_fec_reconstruct_into(ugo_fec* ctx, const uint8_t* shards, const uint64_t* present, size_t groups,
                             size_t shard_size, size_t row_stride, size_t group_stride, uint8_t* out,
                             size_t out_row_stride, size_t out_group_stride, unsigned flags,
                             int8_t* status, void* stream);

/* Reconstruct from a table of row pointers: the rows of a group need not sit
 * in a batch.  Row r of group g is rows[g*(d+p) + r], a DEVICE address
 * (device memory, or pinned host memory through its device mapping -- see
 * ugo_fec_device_address; the kernels then read it over PCIe in place, e.g. a
 * pool of received packet buffers).  Entries of absent rows are not read.
 * Presence, survivors, outputs, flags and status as ugo_fec_reconstruct_into
 * (Encoder.Reconstruct, ugo/fec.go:202, with erased shards nil and filled in
 * fresh buffers): output i of group g -- the i-th erased row, ascending --
 * goes to out + g*out_group_stride + i*out_row_stride, i < p (DATA_ONLY:
 * i < min(d, p), the most data rows a recoverable group can miss).  The
 * survivor rows a group uses must be 16-B aligned and non-null, else that
 * group gets status UGO_FEC_ERR_INVALID_ARG (checked on the device) and is
 * not written; each must be readable for round_up(shard_size, 16) bytes (the
 * kernel loads whole 16-B chunks; bytes past shard_size never reach an
 * output, and output bytes past shard_size are not written).
 * `rows`, `present`, `status`, `out`: device or pinned host memory; out
 * 16-B aligned with strides % 16 == 0; d+p <= 64.  Asynchronous on `stream`.
 * rows[] may be overwritten, and the rows it points to reused, only after
 * the stream has passed this call. */
int ugo_fec_reconstruct_rows(ugo_fec* ctx, const uint8_t* const* rows, const uint64_t* present, size_t groups,
                             size_t shard_size, uint8_t* out, size_t out_row_stride, size_t out_group_stride,
                             unsigned flags, int8_t* status, void* stream);

/* ---- lossy-group list (the recovery ugo's input runs, ugo/fec.go:196-207) --
 * After RX assembly most groups of a batch are complete and need no
 * Reconstruct (input frees them, ugo/fec.go:190-195).  ugo_fec_lossy_groups
 * writes, in ascending order, the index of every group in [0, groups) with an
 * erased row to rebuild -- with UGO_FEC_RECONSTRUCT_DATA_ONLY, an erased DATA
 * row (the groups input calls Reconstruct on; groups with fewer than d shards
 * included, their status says so) -- to list[0 .. *count).  list holds
 * `groups` entries; list, count: device (or pinned) memory; asynchronous on
 * `stream`.  d+p <= 64.
 * ugo_fec_reconstruct_list then runs Reconstruct (ugo/fec.go:202) on the
 * groups list[0 .. *count) of a strided batch: entry j reads group list[j]'s
 * rows; its output i (the i-th erased row in ascending order, erased data rows
 * first; DATA_ONLY: data rows only) goes to
 *     out + j*out_entry_stride + i*out_row_stride
 * (compact: only the lossy groups' recovered shards, in list order, as input
 * returns them), or in place into the batch when out is NULL; status[j] (int8,
 * nullable) as ugo_fec_reconstruct.  The count is read on the device: the
 * call launches for max_entries (<= groups) entries and entries at or past
 * *count do nothing, so no host synchronisation is needed between the two
 * calls.  Code d+p <= 16, 16-B aligned rows and strides (as the fast path). */
int ugo_fec_lossy_groups(ugo_fec* ctx, const uint64_t* present, size_t groups, unsigned flags, uint32_t* list,
                         uint32_t* count, void* stream);
int ugo_fec_reconstruct_list(ugo_fec* ctx, const uint8_t* shards, const uint64_t* present, size_t groups,
                             const uint32_t* list, const uint32_t* count, size_t max_entries,
                             size_t shard_size, size_t row_stride, size_t group_stride, uint8_t* out,
                             size_t out_row_stride, size_t out_entry_stride, unsigned flags, int8_t* status,
                             void* stream);

/* `input`'s recovery over a device batch in one call (ugo/fec.go:190-207):
 * every group with a lost data shard and at least d shards is reconstructed
 * (DATA_ONLY) and its lost data shards are written row-compact, in the order
 * `input` appends them to `recovered` (groups ascending, each group's lost
 * rows ascending): shard r at out + r*out_row_stride, shard_size bytes, for
 * r < min(*count, max_rows) (rows past max_rows are not written), with
 * index[r] = group * (d+p) + row.  *count (device u32) = the number of
 * recovered shards, written on `stream` (no host synchronisation; the
 * lossy-group list and the row offsets are stream-ordered scratch).  A group
 * below d shards recovers nothing, as in `input`.  Code d+p <= 16, 16-B
 * aligned rows and strides (as the fast path); out 16-B aligned,
 * out_row_stride a multiple of 16 >= round_up(shard_size, 16); max_rows = 0
 * counts only (out and index may be NULL). */
int ugo_fec_recover_data(ugo_fec* ctx, const uint8_t* shards, const uint64_t* present, size_t groups,
                         size_t shard_size, size_t row_stride, size_t group_stride, uint8_t* out,
                         size_t out_row_stride, size_t max_rows, uint32_t* index, uint32_t* count, void* stream);

/* The device address of p (device memory of ctx's GPU: p itself; pinned host
 * memory: its device mapping, which on ROCm is the host address), or
 * UGO_FEC_ERR_INVALID_ARG for memory ctx's GPU cannot reach (pageable). */
int ugo_fec_device_address(const ugo_fec* ctx, const void* p, void** dev);

/* ---- host-buffer batch (synchronous) ------------------------------------
 * Same contracts with HOST pointers: the engine stages through its own device
 * buffers, pipelining H2D -> kernel -> D2H over chunks on internal streams.
 * Use ugo_fec_host_alloc() buffers for full-rate DMA.  The reconstruct form
 * returns the first failing group's status (UGO_FEC_OK if none); `status`
 * (host, nullable) receives every group's status. */
int ugo_fec_encode_host(ugo_fec* ctx, uint8_t* shards, size_t groups, size_t shard_size,
                        size_t pitch);
int ugo_fec_reconstruct_host(ugo_fec* ctx, uint8_t* shards, const uint64_t* present,
                             size_t groups, size_t shard_size, size_t pitch, unsigned flags,
                             int8_t* status);

/* ---- per-call latency service --------------------------------------------
 * The drop-in route calls Encode once per group (calcECC, ugo/fec.go:238) and
 * Reconstruct once per lossy group (input, ugo/fec.go:202).  Launched one by
 * one, each call pays a kernel launch and a stream synchronize.  After
 * ugo_fec_service_start, ugo_fec_encode_host / ugo_fec_reconstruct_host calls
 * on PINNED group-major batches of <= 16 groups (shards and pitch multiples of
 * 16; codes with d <= 16, p <= 4, and d + p <= 16 for reconstruct) are served
 * by one resident workgroup polling a mailbox in pinned memory instead: no
 * launch, no synchronize, same bytes and statuses.  The workgroup occupies one
 * CU while it waits; it leaves after `idle_us` (0 = 2000, at most 1000000)
 * without a request and is relaunched by the next call.  Every other call takes the usual path.
 * While it is resident, a device-wide synchronize (hipDeviceSynchronize, and
 * hipFree, which synchronizes the device) waits for it to leave, i.e. up to
 * idle_us after the last call.  Stream work does not: the block runs on a
 * stream of its own priority class, so it has a hardware queue no ordinary
 * stream shares (an ordinary stream placed on its queue would wait).  Those
 * queues are a per-device pool of at most 3 (with GPU_MAX_HW_QUEUES = 4: the
 * process stays within 8 hardware queues); a context that finds the pool
 * leased serves its calls on the launch path.
 * Failure: a call the service cannot complete (a GPU fault, or no answer
 * within the watchdog timeout, 5 s by default) turns the service off, asks the
 * workgroup to leave and waits up to the grace period (5 s by default) for it
 * to be gone, so it can no longer write into the caller's batch; then the call
 * returns UGO_FEC_ERR_HIP and later calls take the launch path.  If the
 * workgroup is still resident after the grace period, the context is
 * POISONED: every later call on it returns UGO_FEC_ERR_HIP, and
 * ugo_fec_destroy frees nothing the workgroup reads (its mailbox and tables
 * are leaked); the caller must then keep the timed-out call's batch alive.
 * ugo_fec_service_stop (and ugo_fec_destroy) waits the same way. */
int ugo_fec_service_start(ugo_fec* ctx, unsigned idle_us);
int ugo_fec_service_stop(ugo_fec* ctx);
/* Watchdog of the service: timeout_ms a call waits for an answer (0 = 5000),
 * grace_ms it then waits for the workgroup to leave (0 = 5000).
 * test_stall_us (tests only; normally 0): the workgroup waits that long before
 * serving each request, from its next launch on, so a test can drive the
 * timeout and poison paths. */
int ugo_fec_service_config(ugo_fec* ctx, unsigned timeout_ms, unsigned grace_ms, unsigned test_stall_us);
/* 1 if the context is poisoned (see above), 0 if not. */
int ugo_fec_poisoned(const ugo_fec* ctx);

/* ---- per-call validation shared with the Go shim ------------------------
 * checkShards(shards, nilok) [klauspost] over a list of n shard lengths:
 * ERR_SHARD_NO_DATA if all are empty, ERR_SHARD_SIZE if a non-empty length
 * differs (or an empty one with nil_ok == 0).  Host-only, no device needed. */
int ugo_fec_check_shards(int n, const size_t* lens, int nil_ok, size_t* shard_size);

/* ---- RX group assembly ----------------------
 * The batch form of what ugo does per packet before Reconstruct:
 * Decrypt (ugo/conn.go:390: a fresh RC4 cipher per packet from a fixed key =
 * XOR with one keystream prefix, `pad`), decode (ugo/fec.go:78-89: LE32 seqid,
 * LE16 flag, payload data[6:]) and the group/slot choice of input
 * (ugo/fec.go:145,175: group = seqid / (d+p), slot = seqid % (d+p)).
 *   wire     packet i at wire + i*slot_stride (slot_stride % 16 == 0,
 *            shards 16-B aligned), lens[i] bytes (uint16).
 *   pad      keystream >= slot_stride bytes, or NULL (no decryption).
 * Every buffer may be device memory or pinned host memory (ugo_fec_host_alloc
 * or registered): pinned buffers are used through their device mapping, so a
 * recvmmsg ring is read over PCIe by the kernel itself (zero-copy) with no
 * separate H2D.  Pageable host memory is rejected (UGO_FEC_ERR_INVALID_ARG).
 * A packet whose flag is typeData (0xf1) or typeFEC (0xf2) and whose group is
 * in [first_group, first_group + groups) is written to row seqid % (d+p) of
 * group seqid/(d+p) - first_group of the strided batch: its payload bytes
 * [0, min(len-6, shard_size)) then zeros up to round_up(shard_size, 16) --
 * whole 16-B chunks, so a row's last chunk also zeroes its bytes past
 * shard_size (each row slot, the batch's last one included, must span
 * round_up(shard_size, 16) bytes; with 16-B strides every slot but the last
 * does); bit row of
 * present[group] is OR-ed (zero `present` before the first call of a batch).
 * stats (device u32[5], nullable) counts accepted / bad-flag / out-of-window /
 * too-short / duplicate packets.  Then ugo_fec_reconstruct_strided recovers
 * the batch.
 *
 * Batch-window rule (what replaces input's per-packet queue, ugo/fec.go:107-226):
 *  - one call is one window of arrivals, in ring order (packet index order);
 *  - dedupe (ugo/fec.go:123-129: a seqid already queued drops the new packet):
 *    for each seqid the FIRST accepted packet in ring order is placed; later
 *    copies -- whatever their payload or length -- count as duplicates and
 *    write nothing.  Deterministic: the same ring gives the same batch;
 *  - expiry (fecExpire, ugo/fec.go:109-121) and the rxlimit trim (:220-224)
 *    bound how long a packet waits for its group.  Here the caller bounds it
 *    by what it puts in a ring and by [first_group, first_group + groups):
 *    packets of groups outside that window are counted out-of-window and
 *    dropped, as a packet older than rxlimit arrivals or fecExpire is;
 *  - the same holds across calls into one batch: a packet whose (group, row)
 *    bit is already set in `present` when the call starts -- placed by an
 *    earlier call -- is a duplicate and writes nothing, so the earlier call's
 *    copy stays, as the queued packet does in input;
 * Placement is optimistic: the extra claim and re-place passes run (inside
 * the call, gated on the device) only when the window holds a duplicate.
 * The engine takes (groups*(8 + (d+p)*4)) bytes of stream-ordered scratch per
 * call (the presence snapshot and the claim words).  npackets < 2^32 - 1. */
int ugo_fec_rx_assemble(ugo_fec* ctx, const uint8_t* wire, size_t slot_stride, const uint16_t* lens,
                        size_t npackets, const uint8_t* pad, uint64_t first_group, size_t groups,
                        uint8_t* shards, size_t shard_size, size_t row_stride, size_t group_stride,
                        uint64_t* present, uint32_t* stats, void* stream);

/* ugo_fec_rx_assemble in the FRAME layout: row seqid % (d+p) of the group
 * receives the decrypted packet itself -- packet bytes [0, min(len,
 * shard_size + 6)), then zeros up to round_up(shard_size + 6, 16) -- instead
 * of its payload: header (LE32 seqid, LE16 flag) in columns 0..5, payload
 * data[6:] in columns 6 .. 6 + shard_size, i.e. the frame ugo's sender keeps
 * (calcECC's window starts at offset 6, ugo/fec.go:228-236, ugo/conn.go:670).
 * Every other rule (flags, window, first copy wins, presence, stats, scratch)
 * as ugo_fec_rx_assemble; each row slot must span round_up(shard_size + 6, 16)
 * bytes.  A packet chunk lands at the offset it was read from, so the kernel
 * needs no byte realignment.  Recovery: run any reconstruct entry point on the
 * frame batch with shard size shard_size + 6.  GF(2^8) columns are
 * independent, so payload columns of a recovered row are bit-identical to the
 * payload-layout result; its columns 0..5 are a combination of the survivors'
 * headers and carry no meaning (a caller reads the shard from column 6). */
int ugo_fec_rx_assemble_frames(ugo_fec* ctx, const uint8_t* wire, size_t slot_stride, const uint16_t* lens,
                               size_t npackets, const uint8_t* pad, uint64_t first_group, size_t groups,
                               uint8_t* shards, size_t shard_size, size_t row_stride, size_t group_stride,
                               uint64_t* present, uint32_t* stats, void* stream);

/* TX group assembly for a batch of `groups` outgoing groups (device or pinned
 * host memory, as for RX; stream-ordered, asynchronous) -- replaces the sender loop ugo/conn.go:643-685
 * (markData, copy into the group buffers, calcECC(group, 6, maxsize),
 * markFEC, ecc[k][:maxsize]) plus crypt.Encrypt (ugo/conn.go:634) per packet:
 *   pkts:   data packet k of group g at pkts + (g*d + k)*slot_in, lens[g*d + k]
 *           bytes (6-B header space first, as markData expects), 6..max_len;
 *   wire:   wire packet r of group g (r < d data, then p parity) at
 *           wire + (g*(d+p) + r)*slot_out, length wire_lens[g*(d+p) + r]:
 *           header (LE32 seqid, LE16 0xf1 / 0xf2), payload or parity over the
 *           window [6, maxsize) of zero-padded group buffers, XOR pad (when not
 *           null: the fixed-key RC4 keystream, >= round_up(max_len, 16) bytes).
 * Seqids run from first_seq (a multiple of d+p below paws, as FEC.next always
 * is at a group boundary) and wrap at paws like markFEC.  A group with a
 * length outside [6, max_len] gets status UGO_FEC_ERR_SHARD_SIZE and
 * wire_lens 0.  A group whose data packets are all header-only (6 bytes) has
 * an empty parity window: as in the sender loop, whose calcECC then fails, its
 * data packets go out and no parity does (status UGO_FEC_ERR_SHARD_NO_DATA,
 * parity wire_lens 0); the batch still spends d+p seqids on it, where the
 * reference's counter would move by d.  slot_in, slot_out: multiples of 16, >= round_up(max_len, 16);
 * d <= 32. */
int ugo_fec_tx_assemble(ugo_fec* ctx, const uint8_t* pkts, size_t slot_in, const uint16_t* lens,
                        size_t groups, uint32_t first_seq, const uint8_t* pad, size_t max_len,
                        uint8_t* wire, size_t slot_out, uint16_t* wire_lens, int8_t* status,
                        void* stream);

/* ---- host-memory RX and TX paths ----------------------------------------
 * The RX path from the socket's receive buffers to the recovered packets, host
 * memory in and out (ugo/listener.go:48 ReadFrom -> Conn.handlePacket,
 * ugo/conn.go:387-406 -> FEC.input, ugo/fec.go:107-226): the packet ring
 * (npackets slots of slot_stride bytes, lens[i] bytes each; host memory,
 * pinned -- ugo_fec_host_alloc -- for full-rate DMA) is copied to the device
 * in chunks that overlap their assembly (ugo_fec_rx_assemble semantics over
 * the window [first_group, first_group + groups), one call per chunk, the first
 * copy of a seqid in ring order wins), then every group with a lost data
 * shard is recovered (ugo_fec_lossy_groups + ugo_fec_reconstruct_list,
 * DATA_ONLY) and only the recovered shards come back, row-compact, in the
 * order ugo's input appends them to `recovered` (ugo/fec.go:203-207: groups
 * ascending, each group's lost data rows ascending; a group with fewer than d
 * shards recovers nothing, as there):
 *   *n_out        the number of recovered data shards;
 *   out + r*out_row_stride: recovered shard r, shard_size bytes, for
 *                 r < min(*n_out, max_out) -- shards past max_out are not
 *                 returned (max_out = 0: no recovery; *n_out still counts them);
 *   out_index[r]  its place: (window group) * (d+p) + row, i.e. its seqid
 *                 minus first_group * (d+p);
 *   present_out   (host u64[groups], nullable) the presence masks after
 *                 assembly; stats_out (host u32[5], nullable) the counts of
 *                 ugo_fec_rx_assemble (set, not added).
 * pad: host memory, >= slot_stride bytes, or NULL.  Synchronous.  d+p <= 16,
 * groups*(d+p) < 2^32.  The device batch ([d+p][groups][round_up(shard_size, 16)]) and the staging
 * are the engine's (stream-ordered scratch). */
int ugo_fec_rx_recover_host(ugo_fec* ctx, const uint8_t* wire, size_t slot_stride, const uint16_t* lens,
                            size_t npackets, const uint8_t* pad, uint64_t first_group, size_t groups,
                            size_t shard_size, uint64_t* present_out, uint32_t* stats_out, uint8_t* out,
                            size_t out_row_stride, size_t max_out, uint32_t* out_index, size_t* n_out);

/* ugo_fec_tx_assemble with every buffer in host memory (pinned for full-rate
 * DMA): the groups go through the device in chunks -- each chunk's data
 * packets H2D, assembled, its wire packets D2H, the three on streams of their
 * own through four device stages, so both copy directions run at once; the
 * lengths go in and the wire lengths and statuses come back with one copy
 * each (ugo_fec_set_tx_host_route: the wire packets written through the
 * buffer's mapping instead).  Same arguments and results (the bytes of a wire
 * slot past its wire_len are unspecified); synchronous. */
int ugo_fec_tx_assemble_host(ugo_fec* ctx, const uint8_t* pkts, size_t slot_in, const uint16_t* lens,
                             size_t groups, uint32_t first_seq, const uint8_t* pad, size_t max_len,
                             uint8_t* wire, size_t slot_out, uint16_t* wire_lens, int8_t* status);

/* The route of ugo_fec_tx_assemble_host's wire packets: 0 = through the
 * device stage and a D2H copy (the default), 1 = written by the kernel through
 * the wire buffer's device mapping, no D2H copy (only when the wire buffer is
 * pinned and 16-B aligned; otherwise the call takes route 0).  Both give the
 * same packets and lengths.  UGO_FEC_ERR_INVALID_ARG for any other value. */
int ugo_fec_set_tx_host_route(ugo_fec* ctx, int route);

/* on = 1 (the default since ABI 9): the host paths' H2D copy stream
 * (ugo_fec_rx_recover_host, ugo_fec_tx_assemble_host, the staged *_host paths)
 * comes from the low-priority stream class, whose hardware queues are a pool of
 * their own, so it never shares one with the context's kernel stream: host TX
 * of 65,536 (10+3) groups runs 26.5-26.6 ms whatever streams the process made
 * before, against 40.1 ms in some process histories with on = 0.  Hardware
 * queues: a process past 8 of them runs oversubscribed (time-sliced), which
 * costs concurrent work ~33 % while a per-call service block is resident; the
 * library keeps its own footprint within 8 -- the normal class, this one low
 * queue, at most 3 service queues with GPU_MAX_HW_QUEUES = 4 -- and an
 * application that adds priority streams of its own should count them
 * (DESIGN.md §6.2).  Synchronizes and replaces the stream when it exists. */
int ugo_fec_set_host_copy_queue(ugo_fec* ctx, int on);

/* RC4 keystream (crypto/rc4 KSA + PRGA) of a key, host memory: the pad above
 * for ugo's fixed-key rc4StreamCrypto (ugo/crypto.go:14-39). */
int ugo_fec_rc4_keystream(const uint8_t* key, size_t key_len, uint8_t* out, size_t n);

/* ---- launch timing (measurement) -----------------------------------------
 * Between ugo_fec_timing_begin and ugo_fec_timing_end, the first max_launches
 * kernels this context launches are issued with hipExtLaunchKernel start/stop
 * events, which take the dispatch's own begin/end timestamps: per-launch
 * kernel durations with nothing inserted into the stream between kernels.
 * timing_end waits for those launches, writes up to `cap` records (launch
 * order) and reports how many launches ran untimed past max_launches. */
#define UGO_FEC_KERNEL_ENCODE 1      /* encode                                  */
#define UGO_FEC_KERNEL_RECONSTRUCT 2 /* reconstruct (descriptor apply)          */
#define UGO_FEC_KERNEL_PREPARE 3     /* per-group decode descriptors (d+p > 16) */
#define UGO_FEC_KERNEL_BYTES 4       /* byte-granular encode / reconstruct      */
#define UGO_FEC_KERNEL_RX 5          /* ugo_fec_rx_assemble                     */
#define UGO_FEC_KERNEL_TX 6          /* ugo_fec_tx_assemble                     */
#define UGO_FEC_KERNEL_PACKET 7      /* ugo_fec_packet_decode                   */

typedef struct ugo_fec_launch_time {
  uint32_t kernel; /* UGO_FEC_KERNEL_* */
  float ms;        /* kernel duration */
} ugo_fec_launch_time;

int ugo_fec_timing_begin(ugo_fec* ctx, size_t max_launches);
int ugo_fec_timing_end(ugo_fec* ctx, ugo_fec_launch_time* out, size_t cap, size_t* n_out,
                       size_t* n_untimed);

/* ---- helpers ------------------------------------------------------------- */
/* pinned host memory */
int ugo_fec_host_alloc(size_t bytes, void** out);
/* tests only (fault injection): pinned allocations of more than `bytes` fail
 * with UGO_FEC_ERR_HIP, as on a host out of pinnable memory; 0 = no limit */
int ugo_fec_set_host_alloc_limit(size_t bytes);
int ugo_fec_host_free(void* p);
const char* ugo_fec_strerror(int status);
int ugo_fec_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* UGO_FEC_H */
