// Package ugofec is the klauspost/reedsolomon Encoder subset jflyup/ugo uses
// (New at ugo/fec.go:59, Reconstruct at :202, Encode at :238), backed by the
// MI355X engine libugofec.so through its C-ABI (include/ugo_fec.h), plus the
// batch RX / TX paths from and to host memory.
//
// Build: make -C ugo_amd/csrc first (-> ugo_amd/libugofec.so).  The cgo flags
// below point at this repository's include/ and ugo_amd/ from go/ugofec; a
// copy placed elsewhere (e.g. next to ugo/ as github.com/jflyup/ugo/ugofec)
// sets CGO_CFLAGS=-I<repo>/include and CGO_LDFLAGS="-L<repo>/ugo_amd
// -lugofec -Wl,-rpath,<repo>/ugo_amd" instead.  go/fec.go.patch is the edit
// to ugo/fec.go that swaps the encoder.
//
// tests/test_cgo_shim_replay.py replays this file's C calls through ctypes
// (the build container has no Go toolchain) and checks that every C.ugo_fec_*
// call below is one it replays.
package ugofec

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#cgo LDFLAGS: -L${SRCDIR}/../../ugo_amd -lugofec -Wl,-rpath,${SRCDIR}/../../ugo_amd
#include <stdlib.h>
#include "ugo_fec.h"
*/
import "C"

import (
	"errors"
	"unsafe"
)

// Same messages as klauspost/reedsolomon, so log output in ugo/fec.go is unchanged.
var (
	ErrInvShardNum  = errors.New("cannot create Encoder with less than one data shard or less than zero parity shards")
	ErrMaxShardNum  = errors.New("cannot create Encoder with more than 256 data+parity shards")
	ErrTooFewShards = errors.New("too few shards given")
	ErrShardNoData  = errors.New("no shard data")
	ErrShardSize    = errors.New("shard sizes do not match")
)

func statusErr(st C.int) error {
	switch st {
	case C.UGO_FEC_OK:
		return nil
	case C.UGO_FEC_ERR_INV_SHARD_NUM:
		return ErrInvShardNum
	case C.UGO_FEC_ERR_MAX_SHARD_NUM:
		return ErrMaxShardNum
	case C.UGO_FEC_ERR_TOO_FEW_SHARDS:
		return ErrTooFewShards
	case C.UGO_FEC_ERR_SHARD_NO_DATA:
		return ErrShardNoData
	case C.UGO_FEC_ERR_SHARD_SIZE:
		return ErrShardSize
	}
	return errors.New(C.GoString(C.ugo_fec_strerror(st)))
}

// Encoder is single-owner, like ugo's FEC (used only from Conn.run).
type Encoder struct {
	ctx    *C.ugo_fec
	d, p   int
	stage  unsafe.Pointer // pinned host staging, reused across calls
	stageN int
}

func New(dataShards, parityShards int) (*Encoder, error) {
	if C.ugo_fec_abi_version() != C.UGO_FEC_ABI_VERSION { // header and library from one build
		return nil, errors.New("libugofec: ABI version mismatch")
	}
	var ctx *C.ugo_fec
	if st := C.ugo_fec_create(0, C.int(dataShards), C.int(parityShards), &ctx); st != C.UGO_FEC_OK {
		return nil, statusErr(st)
	}
	return &Encoder{ctx: ctx, d: dataShards, p: parityShards}, nil
}

func (e *Encoder) Close() {
	poisoned := C.ugo_fec_poisoned(e.ctx) != 0
	C.ugo_fec_destroy(e.ctx) // stops the per-call service too (or leaks what a stuck one reads)
	if e.stage != nil && !poisoned {
		C.ugo_fec_host_free(e.stage)
	}
}

// Optional, once after New: serve the per-group calls below from a resident
// workgroup (ugo_fec_service_start) instead of a kernel launch each --
// Encode 7.0 us and Reconstruct 7.1-7.2 us per call instead of 14-17
// (DESIGN.md §7).  It holds one CU while it waits and leaves after idleUs
// (0 = 2000) without a call; the next call brings it back.
func (e *Encoder) ServiceStart(idleUs uint) error {
	return statusErr(C.ugo_fec_service_start(e.ctx, C.uint(idleUs)))
}

// A call the service cannot complete returns ErrHip only after the workgroup
// has left (it can no longer write the caller's stage); later calls take the
// launch path.  If the workgroup never leaves within the grace period the
// context is poisoned: every call then fails, and Close leaks the mailbox the
// workgroup still reads -- the shim must then also keep e.stage (never free
// a stage a stuck workgroup may still write).
func (e *Encoder) Poisoned() bool { return C.ugo_fec_poisoned(e.ctx) != 0 }

// Go memory may not be retained by C (cgo pointer rules), so shards are
// copied into a pinned staging buffer laid out as one group [d+p][P], rows at
// a 16-byte pitch P = (S+15) &^ 15: the engine's vector kernels need 16-B
// aligned rows, and ugo's shards (1470-B calcECC window, 1476-B input
// buffers) are not multiples of 16 -- at pitch S every call would fall to the
// byte-granular kernel.  Bytes [S, P) of a row are padding the engine never
// writes.
func pitch(S int) int { return (S + 15) &^ 15 }

func (e *Encoder) staging(n int) []byte {
	if n > e.stageN {
		if e.stage != nil {
			C.ugo_fec_host_free(e.stage)
		}
		C.ugo_fec_host_alloc(C.size_t(n), &e.stage)
		e.stageN = n
	}
	return unsafe.Slice((*byte)(e.stage), n)
}

func (e *Encoder) check(shards [][]byte, nilOK bool) (int, error) {
	n := e.d + e.p
	if len(shards) != n {
		return 0, ErrTooFewShards
	}
	lens := make([]C.size_t, n)
	for i, s := range shards {
		lens[i] = C.size_t(len(s))
	}
	var size C.size_t
	ok := C.int(0)
	if nilOK {
		ok = 1
	}
	if st := C.ugo_fec_check_shards(C.int(n), &lens[0], ok, &size); st != C.UGO_FEC_OK {
		return 0, statusErr(st)
	}
	return int(size), nil
}

// Encode: parity shards written in place (ugo/fec.go:238).
func (e *Encoder) Encode(shards [][]byte) error {
	S, err := e.check(shards, false)
	if err != nil {
		return err
	}
	n, P := e.d+e.p, pitch(S)
	buf := e.staging(n * P)
	for k := 0; k < e.d; k++ {
		copy(buf[k*P:k*P+S], shards[k])
	}
	if st := C.ugo_fec_encode_host(e.ctx, (*C.uint8_t)(e.stage), 1, C.size_t(S), C.size_t(P)); st != C.UGO_FEC_OK {
		return statusErr(st)
	}
	for k := e.d; k < n; k++ {
		copy(shards[k], buf[k*P:k*P+S])
	}
	return nil
}

func (e *Encoder) reconstruct(shards [][]byte, flags C.uint) error {
	S, err := e.check(shards, true)
	if err != nil {
		return err
	}
	n, P := e.d+e.p, pitch(S)
	buf := e.staging(n * P)
	var mask [4]C.uint64_t // ceil(n/64) words: upstream allows n <= 256
	for r, s := range shards {
		if len(s) != 0 {
			mask[r/64] |= 1 << uint(r%64)
			copy(buf[r*P:r*P+S], s)
		}
	}
	var status C.int8_t
	if st := C.ugo_fec_reconstruct_host(e.ctx, (*C.uint8_t)(e.stage), &mask[0], 1, C.size_t(S), C.size_t(P),
		flags, &status); st != C.UGO_FEC_OK {
		return statusErr(st)
	}
	limit := n
	if flags&C.UGO_FEC_RECONSTRUCT_DATA_ONLY != 0 {
		limit = e.d
	}
	for r := 0; r < limit; r++ {
		if len(shards[r]) != 0 {
			continue
		}
		if cap(shards[r]) >= S { // upstream: reuse capacity, else allocate
			shards[r] = shards[r][0:S]
		} else {
			shards[r] = make([]byte, S)
		}
		copy(shards[r], buf[r*P:r*P+S])
	}
	return nil
}

// Reconstruct: every missing shard, data and parity (ugo/fec.go:202).
func (e *Encoder) Reconstruct(shards [][]byte) error { return e.reconstruct(shards, 0) }

// ReconstructData: missing data shards only.
func (e *Encoder) ReconstructData(shards [][]byte) error {
	return e.reconstruct(shards, C.UGO_FEC_RECONSTRUCT_DATA_ONLY)
}

// ---- batch paths (host memory in and out; DESIGN.md §6.2) -------------------

// HostAlloc returns n bytes of pinned host memory (full-rate DMA for the ring
// and packet buffers below); free it with HostFree.  Go slices over C memory
// are allowed by the cgo rules, and the engine never retains them past a call.
func HostAlloc(n int) ([]byte, error) {
	var p unsafe.Pointer
	if st := C.ugo_fec_host_alloc(C.size_t(n), &p); st != C.UGO_FEC_OK {
		return nil, statusErr(st)
	}
	return unsafe.Slice((*byte)(p), n), nil
}

func HostFree(b []byte) {
	if len(b) != 0 {
		C.ugo_fec_host_free(unsafe.Pointer(&b[0]))
	}
}

func u8(b []byte) *C.uint8_t {
	if len(b) == 0 {
		return nil
	}
	return (*C.uint8_t)(unsafe.Pointer(&b[0]))
}

// RecoverRing is the receive side for a whole ring of received packets
// (ugo/listener.go:48 -> Conn.handlePacket, ugo/conn.go:387-406 -> FEC.input,
// ugo/fec.go:107-226) in one call (ugo_fec_rx_recover_host): packet i at
// ring[i*slot:], lens[i] bytes; pad = the fixed-key RC4 keystream (>= slot
// bytes) or nil.  Returns n, the number of recovered data shards; the first
// min(n, len(index)) of them are written to out (shard r at out[r*outStride:],
// shardSize bytes) in the order input appends them to `recovered`, with
// index[r] = (group - firstGroup)*(d+p) + row.  stats: accepted, bad flag,
// out of window, too short, duplicate.
func (e *Encoder) RecoverRing(ring []byte, slot int, lens []uint16, pad []byte, firstGroup uint64, groups int,
	shardSize int, out []byte, outStride int, index []uint32) (n int, stats [5]uint32, err error) {
	npk := len(lens)
	maxOut := len(index)
	if maxOut > 0 && len(out) < (maxOut-1)*outStride+shardSize {
		return 0, stats, errors.New("ugofec: out holds fewer than len(index) shards")
	}
	if npk > 0 && len(ring) < npk*slot {
		return 0, stats, errors.New("ugofec: ring holds fewer than len(lens) slots")
	}
	var idx *C.uint32_t
	if maxOut > 0 {
		idx = (*C.uint32_t)(unsafe.Pointer(&index[0]))
	}
	var lp *C.uint16_t
	if npk > 0 {
		lp = (*C.uint16_t)(unsafe.Pointer(&lens[0]))
	}
	var nOut C.size_t
	st := C.ugo_fec_rx_recover_host(e.ctx, u8(ring), C.size_t(slot), lp, C.size_t(npk), u8(pad),
		C.uint64_t(firstGroup), C.size_t(groups), C.size_t(shardSize), nil,
		(*C.uint32_t)(unsafe.Pointer(&stats[0])), u8(out), C.size_t(outStride), C.size_t(maxOut), idx, &nOut)
	return int(nOut), stats, statusErr(st)
}

// AssembleTx is the sender loop (markData, calcECC, markFEC, crypt.Encrypt;
// ugo/conn.go:634, :643-685) for groups groups of d data packets
// (ugo_fec_tx_assemble_host): data packet k of group g at pkts[(g*d+k)*slotIn:],
// lens[g*d+k] bytes with the 6-B header space first; wire packet r of group g
// at wire[(g*(d+p)+r)*slotOut:], wireLens[g*(d+p)+r] bytes, seqids from
// firstSeq.  The caller advances FEC.next by groups*(d+p) (mod paws).
func (e *Encoder) AssembleTx(pkts []byte, slotIn int, lens []uint16, firstSeq uint32, pad []byte, maxLen int,
	wire []byte, slotOut int, wireLens []uint16, status []int8) error {
	n := e.d + e.p
	if len(lens)%e.d != 0 {
		return errors.New("ugofec: lens must hold whole groups of d packets")
	}
	groups := len(lens) / e.d
	if groups == 0 {
		return nil
	}
	if len(pkts) < groups*e.d*slotIn || len(wire) < groups*n*slotOut || len(wireLens) < groups*n ||
		(status != nil && len(status) < groups) {
		return errors.New("ugofec: buffer shorter than the batch")
	}
	var sp *C.int8_t
	if status != nil {
		sp = (*C.int8_t)(unsafe.Pointer(&status[0]))
	}
	return statusErr(C.ugo_fec_tx_assemble_host(e.ctx, u8(pkts), C.size_t(slotIn),
		(*C.uint16_t)(unsafe.Pointer(&lens[0])), C.size_t(groups), C.uint32_t(firstSeq), u8(pad), C.size_t(maxLen),
		u8(wire), C.size_t(slotOut), (*C.uint16_t)(unsafe.Pointer(&wireLens[0])), sp))
}
