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
	reserve(shards)
	v := newShardVec(shards)
	defer v.free()
	st := C.cfsec_ec_encode(e.h, v.ptr(), C.int(v.n), C.CFSEC_MEM_HOST, nil)
	v.lens(shards)
	return ecError(st)
}

func badVec(badIdx []int) ([]C.int, *C.int) {
	if len(badIdx) == 0 {
		return nil, nil
	}
	b := make([]C.int, len(badIdx))
	for i, v := range badIdx {
		b[i] = C.int(v)
	}
	return b, &b[0]
}

func (e *ECEncoder) reconstruct(shards [][]byte, badIdx []int, dataOnly bool) error {
	// initBadShards (encoder.go:182-188) happens in C; a bad shard keeps its buffer as capacity
	for _, i := range badIdx {
		if i >= 0 && i < len(shards) && len(shards[i]) != 0 {
			shards[i] = shards[i][:0]
		}
	}
	reserve(shards)
	v := newShardVec(shards)
	defer v.free()
	b, bp := badVec(badIdx)
	var pin runtime.Pinner
	if bp != nil {
		pin.Pin(bp)
	}
	defer pin.Unpin()
	var st C.int
	if dataOnly {
		st = C.cfsec_ec_reconstruct_data(e.h, v.ptr(), C.int(v.n), bp, C.int(len(b)), C.CFSEC_MEM_HOST, nil)
	} else {
		st = C.cfsec_ec_reconstruct(e.h, v.ptr(), C.int(v.n), bp, C.int(len(b)), C.CFSEC_MEM_HOST, nil)
	}
	v.lens(shards)
	return ecError(st)
}

func (e *ECEncoder) Reconstruct(shards [][]byte, badIdx []int) error {
	return e.reconstruct(shards, badIdx, false)
}

func (e *ECEncoder) ReconstructData(shards [][]byte, badIdx []int) error {
	return e.reconstruct(shards, badIdx, true)
}

func (e *ECEncoder) Verify(shards [][]byte) (bool, error) {
	v := newShardVec(shards)
	defer v.free()
	var ok C.int
	err := ecError(C.cfsec_ec_verify(e.h, v.ptr(), C.int(v.n), C.CFSEC_MEM_HOST, nil, &ok))
	return ok != 0, err
}

// ReconstructBatch runs blobnode's repair step (work_shard_recover.go:751-760) for a whole tasklet:
// for every bid, Reconstruct(bids[b], badIdx[b]) then, with verify, Verify(bids[b]) -- one call,
// one fused pass per bid (LRC: one pass too when no local shard is bad, else the global pass then
// the AZ-local pass).  errs[b] is what that bid's
// two calls would have reported (ErrVerify for a false Verify); err reports a failure of the call
// itself.  Zero-size bids are skipped by the caller, as the reference loop does (:730-733).
func (e *ECEncoder) ReconstructBatch(bids [][][]byte, badIdx [][]int, verify bool) (errs []error, err error) {
	if len(bids) != len(badIdx) {
		return nil, errInvalidArg
	}
	errs = make([]error, len(bids))
	if len(bids) == 0 {
		return errs, nil
	}
	n := len(bids[0])
	flat := make([][]byte, 0, n*len(bids))
	var bad []C.int
	off := make([]C.int, 1, len(bids)+1)
	for b, shards := range bids {
		if len(shards) != n {
			return nil, errInvalidArg
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
	v := newShardVec(flat)
	defer v.free()
	status := make([]C.int, len(bids))
	var pin runtime.Pinner
	defer pin.Unpin()
	pin.Pin(&status[0])
	pin.Pin(&off[0])
	var bp *C.int
	if len(bad) > 0 {
		pin.Pin(&bad[0])
		bp = &bad[0]
	}
	vf := C.int(0)
	if verify {
		vf = 1
	}
	st := C.cfsec_ec_reconstruct_batch(e.h, v.ptr(), C.int(n), C.int(len(bids)), bp, &off[0], vf,
		C.CFSEC_MEM_HOST, &status[0])
	v.lens(flat)
	for b := range bids {
		copy(bids[b], flat[b*n:(b+1)*n])
		errs[b] = ecError(status[b])
	}
	return errs, toError(st)
}

// RepairRows returns the first N present global shards a Reconstruct decodes from with badIdx lost
// (KRS/reedsolomon.go:1453-1465) and, for every wanted shard index (data, global or LRC local
// parity), its GF(2^8) row over them (cfsec_ec_repair_rows): the repair plan of survivors that
// live elsewhere, e.g. on other GPUs.
func (e *ECEncoder) RepairRows(badIdx, want []int) (in []int, rows [][]byte, err error) {
	n := e.tactic.N
	_, pbad := badVec(badIdx) // the pointer passed to C keeps the slice alive for the call
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
	// lrcencoder.go:203-222: the local shards follow in the same buffer when it has room
	shardN, shardLen := len(shards), len(shards[0])
	if cap(data) >= (e.tactic.L+shardN)*shardLen {
		if cap(data) > len(data) {
			data = data[:cap(data)]
		}
		for i := 0; i < e.tactic.L; i++ {
			shards = append(shards, data[(shardN+i)*shardLen:(shardN+i+1)*shardLen])
		}
	} else {
		for i := 0; i < e.tactic.L; i++ {
			shards = append(shards, make([]byte, shardLen))
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
