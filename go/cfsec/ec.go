package cfsec

/*
#include <stdlib.h>
#include "cfsec.h"
*/
import "C"

import (
	"errors"
	"io"
	"runtime"
	"unsafe"

	"github.com/cubefs/cubefs/blobstore/common/codemode"
	"github.com/klauspost/reedsolomon"
)

// ECEncoder implements CubeFS's ec.Encoder (blobstore/common/ec/encoder.go:41-62) whole, over the
// cfsec_ec_* entry points: the LRC modes take the fused (M+L) x N encode (one launch instead of a
// global Encode, one local Encode per AZ and, with EnableVerify, three Verifies -- lrcencoder.go:
// 35-82), and blobnode's repair loop can hand over a whole tasklet (ReconstructBatch).
// The sentinel errors are ec's own (encoder.go:33-38); a copy of this file dropped into package
// ec returns those variables instead of the ones below.
type ECEncoder struct {
	h      *C.cfsec_ec
	tactic codemode.Tactic
	engine *Engine // Split / Join (host bookkeeping)
}

var (
	ErrShortData       = errors.New("short data")
	ErrInvalidCodeMode = errors.New("invalid code mode")
	ErrVerify          = errors.New("shards verify failed")
	ErrInvalidShards   = errors.New("invalid shards")
)

func ecError(st C.int) error {
	switch st {
	case C.CFSEC_ERR_INVALID_CODE_MODE:
		return ErrInvalidCodeMode
	case C.CFSEC_ERR_VERIFY:
		return ErrVerify
	case C.CFSEC_ERR_INVALID_SHARDS:
		return ErrInvalidShards
	case C.CFSEC_ERR_SHORT_DATA:
		return ErrShortData
	default:
		return toError(st)
	}
}

// NewECEncoder mirrors ec.NewEncoder(Config{CodeMode, EnableVerify, Concurrency}) (encoder.go:78-112).
func NewECEncoder(t codemode.Tactic, enableVerify bool, concurrency int) (*ECEncoder, error) {
	if !t.IsValid() {
		return nil, ErrInvalidCodeMode
	}
	ct := C.cfsec_tactic{n: C.int(t.N), m: C.int(t.M), l: C.int(t.L), az_count: C.int(t.AZCount),
		put_quorum: C.int(t.PutQuorum), get_quorum: C.int(t.GetQuorum), min_shard_size: C.int(t.MinShardSize)}
	ev := C.int(0)
	if enableVerify {
		ev = 1
	}
	var h *C.cfsec_ec
	if err := ecError(C.cfsec_ec_new(&ct, ev, C.int(concurrency), -1, &h)); err != nil {
		return nil, err
	}
	eng, err := New(t.N, t.M)
	if err != nil {
		C.cfsec_ec_free(h)
		return nil, err
	}
	e := &ECEncoder{h: h, tactic: t, engine: eng}
	runtime.SetFinalizer(e, func(e *ECEncoder) { C.cfsec_ec_free(e.h) })
	return e, nil
}

// SetDevices spreads batches over these HIP devices (cfsec_ec_set_devices).
func (e *ECEncoder) SetDevices(devices []int) error {
	if len(devices) == 0 {
		return errInvalidArg
	}
	d := make([]C.int, len(devices))
	for i, v := range devices {
		d[i] = C.int(v)
	}
	return toError(C.cfsec_ec_set_devices(e.h, &d[0], C.int(len(d))))
}

func intPtr(v []C.int) *C.int {
	if len(v) == 0 {
		return nil
	}
	return &v[0]
}

// reserve gives every zero-length shard capacity for the shard size, as ec.fillFullShards and
// KRS/reedsolomon.go:1514-1518 allocate when cap is short (the C side writes into cap only).
func reserve(shards [][]byte) {
	size := 0
	for _, s := range shards {
		if len(s) != 0 {
			size = len(s)
			break
		}
	}
	if size == 0 {
		return
	}
	for i, s := range shards {
		if len(s) == 0 && cap(s) < size {
			shards[i] = reedsolomon.AllocAligned(1, size)[0][:0]
		}
	}
}

func (e *ECEncoder) Encode(shards [][]byte) error {
	if base, size, stride, ok := stripeOf(shards); ok {
		return ecError(C.cfsec_ec_encode_contig(e.h, base, C.size_t(size), C.size_t(stride), C.int(len(shards)),
			C.CFSEC_MEM_HOST, nil))
	}
	reserve(shards)
	return ecError(callVec(shards, func(v *C.cfsec_shard, n C.int) C.int {
		return C.cfsec_ec_encode(e.h, v, n, C.CFSEC_MEM_HOST, nil)
	}))
}

func (e *ECEncoder) reconstruct(shards [][]byte, badIdx []int, dataOnly bool) error {
	donly := C.int(0)
	if dataOnly {
		donly = 1
	}
	b, bp := cints(badIdx)
	// blobnode and access hand over full-length shards of one ec.Buffer with the broken ones named
	// in badIdx: one pointer, rebuilt in place
	if base, size, stride, ok := stripeOf(shards); ok {
		err := ecError(C.cfsec_ec_reconstruct_contig(e.h, base, C.size_t(size), C.size_t(stride), C.int(len(shards)),
			bp, C.int(len(b)), donly, C.CFSEC_MEM_HOST, nil))
		e.contigHeaders(shards, badIdx, dataOnly, err != nil)
		return err
	}
	// initBadShards (encoder.go:182-188) happens in C; a bad shard keeps its buffer as capacity
	for _, i := range badIdx {
		if i >= 0 && i < len(shards) && len(shards[i]) != 0 {
			shards[i] = shards[i][:0]
		}
	}
	if e.tactic.L == 0 {
		// RS modes: the engine's Reconstruct allocates only the shards it rebuilds (encoder.go:139-151)
		prepareMissing(shards, e.tactic.N, dataOnly)
	} else {
		// LRC modes: fillFullShards (encoder.go:199-210) gives every zero-length shard the size first
		reserve(shards)
	}
	return ecError(callVec(shards, func(v *C.cfsec_shard, n C.int) C.int {
		if dataOnly {
			return C.cfsec_ec_reconstruct_data(e.h, v, n, bp, C.int(len(b)), C.CFSEC_MEM_HOST, nil)
		}
		return C.cfsec_ec_reconstruct(e.h, v, n, bp, C.int(len(b)), C.CFSEC_MEM_HOST, nil)
	}))
}

// contigHeaders leaves the Go headers of a contiguous-stripe reconstruct (rebuilt in place in C,
// every header still the shard size) as the reference leaves them: initBadShards (encoder.go:
// 182-188) cuts every bad global shard to len 0 and the engine's Reconstruct restores the ones it
// rebuilds -- so a bad parity shard of ReconstructData (encoder.go:146-151, lrcencoder.go:188-201)
// and every bad global shard of a failed call keep len 0.  LRC local shards are rebuilt through
// header copies (lrcencoder.go:172-178, 236-243): the caller's keep their length.  A contiguous
// stripe has one shard size, so a failed call failed in the global pass (ErrTooFewShards).
func (e *ECEncoder) contigHeaders(shards [][]byte, badIdx []int, dataOnly, failed bool) {
	N, M := e.tactic.N, e.tactic.M
	for _, i := range badIdx {
		if i < 0 || i >= len(shards) || (e.tactic.L != 0 && i >= N+M) {
			continue
		}
		if failed || (dataOnly && i >= N) {
			shards[i] = shards[i][:0]
		}
	}
}

func (e *ECEncoder) Reconstruct(shards [][]byte, badIdx []int) error {
	return e.reconstruct(shards, badIdx, false)
}

func (e *ECEncoder) ReconstructData(shards [][]byte, badIdx []int) error {
	return e.reconstruct(shards, badIdx, true)
}

func (e *ECEncoder) Verify(shards [][]byte) (bool, error) {
	ok := make([]C.int, 1)
	if base, size, stride, contig := stripeOf(shards); contig {
		err := ecError(C.cfsec_ec_verify_contig(e.h, base, C.size_t(size), C.size_t(stride), C.int(len(shards)),
			C.CFSEC_MEM_HOST, nil, &ok[0]))
		return ok[0] != 0, err
	}
	err := ecError(callVec(shards, func(v *C.cfsec_shard, n C.int) C.int {
		return C.cfsec_ec_verify(e.h, v, n, C.CFSEC_MEM_HOST, nil, &ok[0])
	}))
	return ok[0] != 0, err
}

// ReconstructBatch runs blobnode's repair step (work_shard_recover.go:751-760) for a whole tasklet:
// for every bid, Reconstruct(bids[b], badIdx[b]) then, with verify, Verify(bids[b]) -- one call,
// one fused pass per bid (LRC: one pass too when no local shard is bad, else the global pass then
// the AZ-local pass).  errs[b] is what that bid's two calls would have reported (ErrVerify for a
// false Verify); err reports a failure of the call itself.  Zero-size bids are skipped by the
// caller, as the reference loop does (:730-733).
func (e *ECEncoder) ReconstructBatch(bids [][][]byte, badIdx [][]int, verify bool) (errs []error, err error) {
	errs, _, err = e.reconstructBatch(bids, badIdx, verify, false)
	return errs, err
}

// ReconstructBatchCRC is ReconstructBatch returning, per bid, crc32.ChecksumIEEE of every shard it
// rebuilt (0 for the others and for failed bids): the ShardCrc32 blobnode stores with each repaired
// shard (work_shard_recover.go:335-342), computed on the GPU before the shard leaves HBM.
func (e *ECEncoder) ReconstructBatchCRC(bids [][][]byte, badIdx [][]int, verify bool) ([]error, [][]uint32, error) {
	return e.reconstructBatch(bids, badIdx, verify, true)
}

func (e *ECEncoder) reconstructBatch(bids [][][]byte, badIdx [][]int, verify, wantCRC bool) ([]error, [][]uint32, error) {
	if len(bids) != len(badIdx) {
		return nil, nil, errInvalidArg
	}
	errs := make([]error, len(bids))
	if len(bids) == 0 {
		return errs, nil, nil
	}
	n := len(bids[0])
	flat := make([][]byte, 0, n*len(bids))
	var bad []C.int
	off := make([]C.int, 1, len(bids)+1)
	for b, shards := range bids {
		if len(shards) != n {
			return nil, nil, errInvalidArg
		}
		for _, i := range badIdx[b] {
			if i >= 0 && i < n && len(shards[i]) != 0 {
				shards[i] = shards[i][:0]
			}
			bad = append(bad, C.int(i))
		}
		reserve(shards)
		flat = append(flat, shards...)
		off = append(off, C.int(len(bad)))
	}
	bp := intPtr(bad)
	status := make([]C.int, len(bids))
	words := make([]C.uint32_t, len(bids)*n+1)
	vf := C.int(0)
	if verify {
		vf = 1
	}
	st := callVec(flat, func(v *C.cfsec_shard, _ C.int) C.int {
		if wantCRC {
			return C.cfsec_ec_reconstruct_batch_crc(e.h, v, C.int(n), C.int(len(bids)), bp, &off[0], vf,
				C.CFSEC_MEM_HOST, &status[0], &words[0])
		}
		return C.cfsec_ec_reconstruct_batch(e.h, v, C.int(n), C.int(len(bids)), bp, &off[0], vf,
			C.CFSEC_MEM_HOST, &status[0])
	})
	var crcs [][]uint32
	if wantCRC {
		crcs = make([][]uint32, len(bids))
	}
	for b := range bids {
		copy(bids[b], flat[b*n:(b+1)*n])
		errs[b] = ecError(status[b])
		if wantCRC {
			crcs[b] = make([]uint32, n)
			for i := range crcs[b] {
				crcs[b][i] = uint32(words[b*n+i])
			}
		}
	}
	return errs, crcs, toError(st)
}

// EncodeBatch is access's Put over a batch of blobs (stream_put.go:104-143 encodes them one by one):
// every stripe Encoded as Encode would (EnableVerify included; the LRC modes as one fused pass) in
// one call; errs[s] is what Encode(stripes[s]) would have returned.
func (e *ECEncoder) EncodeBatch(stripes [][][]byte) (errs []error, err error) {
	errs, _, err = e.encodeBatch(stripes, false)
	return errs, err
}

// EncodeBatchCRC is EncodeBatch returning crc32.ChecksumIEEE of every shard of every stripe -- the
// checksums access takes right after encoding (stream_put.go:249-253) -- from the GPU.
func (e *ECEncoder) EncodeBatchCRC(stripes [][][]byte) ([]error, [][]uint32, error) {
	return e.encodeBatch(stripes, true)
}

func (e *ECEncoder) encodeBatch(stripes [][][]byte, wantCRC bool) ([]error, [][]uint32, error) {
	errs := make([]error, len(stripes))
	if len(stripes) == 0 {
		return errs, nil, nil
	}
	n := len(stripes[0])
	flat := make([][]byte, 0, n*len(stripes))
	for _, shards := range stripes {
		if len(shards) != n {
			return nil, nil, errInvalidArg
		}
		reserve(shards)
		flat = append(flat, shards...)
	}
	status := make([]C.int, len(stripes))
	words := make([]C.uint32_t, len(stripes)*n+1)
	st := callVec(flat, func(v *C.cfsec_shard, _ C.int) C.int {
		if wantCRC {
			return C.cfsec_ec_encode_batch_crc(e.h, v, C.int(n), C.int(len(stripes)), C.CFSEC_MEM_HOST, &status[0],
				&words[0])
		}
		return C.cfsec_ec_encode_batch(e.h, v, C.int(n), C.int(len(stripes)), C.CFSEC_MEM_HOST, &status[0])
	})
	var crcs [][]uint32
	if wantCRC {
		crcs = make([][]uint32, len(stripes))
	}
	for s := range stripes {
		copy(stripes[s], flat[s*n:(s+1)*n])
		errs[s] = ecError(status[s])
		if wantCRC {
			crcs[s] = make([]uint32, n)
			for i := range crcs[s] {
				crcs[s][i] = uint32(words[s*n+i])
			}
		}
	}
	return errs, crcs, toError(st)
}

// EncodeBuffer encodes nstripes stripes that live in one allocation (stripe s at s*stripeStride,
// its shards at s*stripeStride + i*stride, shardSize bytes each): one Go pointer for the whole batch
// (cfsec_ec_encode_batch_contig), so it is legal on every Go release with no staging copy.  With
// wantCRC it also returns every shard's checksum.
func (e *ECEncoder) EncodeBuffer(buf []byte, shardSize, stride, stripeStride, nstripes int, wantCRC bool) ([]error, [][]uint32, error) {
	n := e.tactic.N + e.tactic.M + e.tactic.L
	if nstripes <= 0 || shardSize <= 0 || stride < shardSize || len(buf) < (nstripes-1)*stripeStride+(n-1)*stride+shardSize {
		return nil, nil, errInvalidArg
	}
	status := make([]C.int, nstripes)
	words := make([]C.uint32_t, nstripes*n)
	var wp *C.uint32_t
	if wantCRC {
		wp = &words[0]
	}
	st := C.cfsec_ec_encode_batch_contig(e.h, (*C.uint8_t)(unsafe.Pointer(&buf[0])), C.size_t(shardSize), C.size_t(stride),
		C.size_t(stripeStride), C.int(n), C.int(nstripes), C.CFSEC_MEM_HOST, &status[0], wp)
	errs := make([]error, nstripes)
	var crcs [][]uint32
	for s := range errs {
		errs[s] = ecError(status[s])
		if wantCRC {
			c := make([]uint32, n)
			for i := range c {
				c[i] = uint32(words[s*n+i])
			}
			crcs = append(crcs, c)
		}
	}
	return errs, crcs, toError(st)
}

// RepairBuffer is ReconstructBatch[CRC] for a tasklet whose bids live in one allocation: bid b at
// bidOff[b], its n shards packed at its own shard size bidSize[b] (cfsec_ec_reconstruct_batch_contig).
func (e *ECEncoder) RepairBuffer(buf []byte, bidOff, bidSize []uint64, badIdx [][]int, verify, wantCRC bool) ([]error, [][]uint32, error) {
	n := e.tactic.N + e.tactic.M + e.tactic.L
	nb := len(bidOff)
	if nb == 0 || len(bidSize) != nb || len(badIdx) != nb || len(buf) == 0 {
		return nil, nil, errInvalidArg
	}
	for b := range bidOff {
		if bidOff[b]+uint64(n)*bidSize[b] > uint64(len(buf)) {
			return nil, nil, errInvalidArg
		}
	}
	var bad []C.int
	off := []C.int{0}
	for _, bb := range badIdx {
		for _, i := range bb {
			bad = append(bad, C.int(i))
		}
		off = append(off, C.int(len(bad)))
	}
	status := make([]C.int, nb)
	words := make([]C.uint32_t, nb*n)
	var wp *C.uint32_t
	if wantCRC {
		wp = &words[0]
	}
	vf := C.int(0)
	if verify {
		vf = 1
	}
	st := C.cfsec_ec_reconstruct_batch_contig(e.h, (*C.uint8_t)(unsafe.Pointer(&buf[0])),
		(*C.uint64_t)(unsafe.Pointer(&bidOff[0])), (*C.uint64_t)(unsafe.Pointer(&bidSize[0])), C.int(n), C.int(nb),
		intPtr(bad), &off[0], vf, C.CFSEC_MEM_HOST, &status[0], wp)
	errs := make([]error, nb)
	var crcs [][]uint32
	for b := range errs {
		errs[b] = ecError(status[b])
		if wantCRC {
			c := make([]uint32, n)
			for i := range c {
				c[i] = uint32(words[b*n+i])
			}
			crcs = append(crcs, c)
		}
	}
	return errs, crcs, toError(st)
}

// RepairRows returns the first N present global shards a Reconstruct decodes from with badIdx lost
// (KRS/reedsolomon.go:1453-1465) and, for every wanted shard index (data, global or LRC local
// parity), its GF(2^8) row over them (cfsec_ec_repair_rows): the repair plan of survivors that
// live elsewhere, e.g. on other GPUs.
func (e *ECEncoder) RepairRows(badIdx, want []int) (in []int, rows [][]byte, err error) {
	n := e.tactic.N
	_, pbad := cints(badIdx) // the pointer passed to C keeps the slice alive for the call
	w := make([]C.int, len(want)+1)
	for i, v := range want {
		w[i] = C.int(v)
	}
	ci := make([]C.int, n)
	flat := make([]byte, n*len(want)+1)
	st := C.cfsec_ec_repair_rows(e.h, pbad, C.int(len(badIdx)), &w[0], C.int(len(want)), &ci[0],
		(*C.uint8_t)(unsafe.Pointer(&flat[0])))
	if st != C.CFSEC_OK {
		return nil, nil, ecError(st)
	}
	in = make([]int, n)
	for i := range in {
		in[i] = int(ci[i])
	}
	rows = make([][]byte, len(want))
	for r := range rows {
		rows[r] = append([]byte(nil), flat[r*n:(r+1)*n]...)
	}
	return in, rows, nil
}

// ---- host bookkeeping, as encoder.go / lrcencoder.go ----

func (e *ECEncoder) Split(data []byte) ([][]byte, error) {
	shards, err := e.engine.Split(data)
	if err != nil || e.tactic.L == 0 {
		return shards, err
	}
	// lrcencoder.go:203-222: the L local shards take the next L shard-sized pieces of data's
	// capacity when all of them fit there, else fresh zeroed buffers
	n, size := len(shards), len(shards[0])
	room := cap(data) >= (n+e.tactic.L)*size
	whole := data[:cap(data)]
	for i := n; i < n+e.tactic.L; i++ {
		if room {
			shards = append(shards, whole[i*size:(i+1)*size])
		} else {
			shards = append(shards, make([]byte, size))
		}
	}
	return shards, nil
}

func (e *ECEncoder) GetDataShards(shards [][]byte) [][]byte { return shards[:e.tactic.N] }

func (e *ECEncoder) GetParityShards(shards [][]byte) [][]byte {
	if e.tactic.L == 0 {
		return shards[e.tactic.N:]
	}
	return shards[e.tactic.N : e.tactic.N+e.tactic.M]
}

func (e *ECEncoder) GetLocalShards(shards [][]byte) [][]byte {
	if e.tactic.L == 0 {
		return nil
	}
	return shards[e.tactic.N+e.tactic.M:]
}

func (e *ECEncoder) GetShardsInIdc(shards [][]byte, idx int) [][]byte {
	if e.tactic.L == 0 {
		// encoder.go:169-176, the append aliasing included
		n, m, az := e.tactic.N, e.tactic.M, e.tactic.AZCount
		ln, lm := n/az, m/az
		return append(shards[idx*ln:(idx+1)*ln], shards[n+lm*idx:n+lm*(idx+1)]...)
	}
	// lrcencoder.go:236-243
	idxs := make([]C.int, 64)
	var cnt C.int
	if toError(C.cfsec_ec_shards_in_idc(e.h, C.int(idx), &idxs[0], C.int(len(idxs)), &cnt)) != nil {
		return nil
	}
	out := make([][]byte, int(cnt))
	for i := range out {
		out[i] = shards[int(idxs[i])]
	}
	return out
}

func (e *ECEncoder) Join(dst io.Writer, shards [][]byte, outSize int) error {
	if e.tactic.L != 0 {
		shards = shards[:e.tactic.N+e.tactic.M]
	}
	return e.engine.Join(dst, shards, outSize)
}
