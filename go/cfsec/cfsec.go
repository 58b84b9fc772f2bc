// Package cfsec is the cgo binding a CubeFS maintainer drops into
// blobstore/common/ec to run the EC engine on MI355X GPUs.
//
// It implements github.com/klauspost/reedsolomon.Encoder (the seam that
// blobstore/common/ec/encoder.go:86 and :95 construct) over the C ABI in
// include/cfsec.h.  The six methods CubeFS calls -- Encode, Verify, Reconstruct,
// ReconstructData, Split, Join -- go to libcfsec.so; EncodeIdx, ReconstructSome
// and Update, which CubeFS never calls, return reedsolomon.ErrNotSupported.
//
// Source only: this container has no Go toolchain, so the package is not built or
// tested here (see INTEGRATION.md for the build line and the test plan).
package cfsec

/*
#cgo CFLAGS: -I${SRCDIR}/../../include
#cgo LDFLAGS: -L${SRCDIR}/../../chubaofs_amd -lcfsec -Wl,-rpath,${SRCDIR}/../../chubaofs_amd
#include <stdlib.h>
#include "cfsec.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"io"
	"runtime"
	"unsafe"

	"github.com/klauspost/reedsolomon"
)

// Engine is a reedsolomon.Encoder whose arithmetic runs on a GPU.
type Engine struct {
	h            *C.cfsec_rs
	dataShards   int
	parityShards int
}

var _ reedsolomon.Encoder = (*Engine)(nil)

// ErrDevice reports a HIP runtime failure (no device, out of memory, ...).
var ErrDevice = errors.New("cfsec: device error")

var errInvalidArg = errors.New("cfsec: invalid argument")

// toError maps cfsec_status codes back onto the Go sentinels (include/cfsec.h).
func toError(st C.int) error {
	switch st {
	case C.CFSEC_OK:
		return nil
	case C.CFSEC_ERR_TOO_FEW_SHARDS:
		return reedsolomon.ErrTooFewShards
	case C.CFSEC_ERR_SHARD_NO_DATA:
		return reedsolomon.ErrShardNoData
	case C.CFSEC_ERR_SHARD_SIZE:
		return reedsolomon.ErrShardSize
	case C.CFSEC_ERR_INV_SHARD_NUM:
		return reedsolomon.ErrInvShardNum
	case C.CFSEC_ERR_MAX_SHARD_NUM:
		return reedsolomon.ErrMaxShardNum
	case C.CFSEC_ERR_SHORT_DATA:
		return reedsolomon.ErrShortData
	case C.CFSEC_ERR_RECONSTRUCT_REQUIRED:
		return reedsolomon.ErrReconstructRequired
	case C.CFSEC_ERR_NOT_SUPPORTED:
		return reedsolomon.ErrNotSupported
	case C.CFSEC_ERR_DEVICE:
		return fmt.Errorf("%w: %s", ErrDevice, C.GoString(C.cfsec_last_error()))
	case C.CFSEC_ERR_SINGULAR:
		return errors.New("matrix is singular")
	default:
		return fmt.Errorf("%w: %s", errInvalidArg, C.GoString(C.cfsec_status_name(st)))
	}
}

// New mirrors reedsolomon.New(dataShards, parityShards) with default options.
func New(dataShards, parityShards int) (*Engine, error) {
	var h *C.cfsec_rs
	if err := toError(C.cfsec_rs_new(C.int(dataShards), C.int(parityShards), -1, &h)); err != nil {
		return nil, err
	}
	e := &Engine{h: h, dataShards: dataShards, parityShards: parityShards}
	runtime.SetFinalizer(e, func(e *Engine) { C.cfsec_rs_free(e.h) })
	return e, nil
}

// shardVec pins the caller's byte slices and lays them out as a C cfsec_shard array.
// The C side never keeps a pointer after the call returns.
type shardVec struct {
	pin runtime.Pinner
	arr *C.cfsec_shard
	n   int
}

func newShardVec(shards [][]byte) *shardVec {
	v := &shardVec{n: len(shards)}
	if v.n == 0 {
		return v
	}
	v.arr = (*C.cfsec_shard)(C.malloc(C.size_t(v.n) * C.size_t(unsafe.Sizeof(C.cfsec_shard{}))))
	elems := unsafe.Slice(v.arr, v.n)
	for i, s := range shards {
		elems[i] = C.cfsec_shard{data: nil, len: C.size_t(len(s)), cap: C.size_t(cap(s))}
		if cap(s) > 0 {
			p := &s[:cap(s)][0]
			v.pin.Pin(p)
			elems[i].data = (*C.uint8_t)(unsafe.Pointer(p))
		}
	}
	return v
}

func (v *shardVec) ptr() *C.cfsec_shard { return v.arr }

// lens copies the lengths the engine left in the headers back into the Go slices.
func (v *shardVec) lens(shards [][]byte) {
	if v.n == 0 {
		return
	}
	for i, e := range unsafe.Slice(v.arr, v.n) {
		if int(e.len) != len(shards[i]) {
			shards[i] = shards[i][:int(e.len)]
		}
	}
}

func (v *shardVec) free() {
	if v.arr != nil {
		C.free(unsafe.Pointer(v.arr))
	}
	v.pin.Unpin()
}

func (e *Engine) Encode(shards [][]byte) error {
	v := newShardVec(shards)
	defer v.free()
	return toError(C.cfsec_rs_encode(e.h, v.ptr(), C.int(v.n), C.CFSEC_MEM_HOST, nil))
}

// EncodeCRC is Encode followed by crc32.ChecksumIEEE of every shard -- what access computes
// right after encoding (blobstore/access/stream_put.go:249-253) -- in one fused GPU pass.
func (e *Engine) EncodeCRC(shards [][]byte) ([]uint32, error) {
	v := newShardVec(shards)
	defer v.free()
	crcs := make([]uint32, v.n)
	if v.n == 0 {
		return crcs, toError(C.cfsec_rs_encode(e.h, v.ptr(), 0, C.CFSEC_MEM_HOST, nil))
	}
	var pin runtime.Pinner
	pin.Pin(&crcs[0])
	defer pin.Unpin()
	err := toError(C.cfsec_rs_encode_crc(e.h, v.ptr(), C.int(v.n), C.CFSEC_MEM_HOST, nil,
		(*C.uint32_t)(unsafe.Pointer(&crcs[0]))))
	return crcs, err
}

// HostAlloc returns size bytes of page-locked C memory (cfsec_host_alloc) as a byte slice: the
// allocation hook for resourcepool.NewMemPoolWith (common/resourcepool/mempool.go:60), so
// ec.Buffer shards are coded in place over PCIe.  Release it with HostFree.
func HostAlloc(size int) ([]byte, error) {
	if size <= 0 {
		return nil, nil
	}
	var p unsafe.Pointer
	if err := toError(C.cfsec_host_alloc(C.size_t(size), &p)); err != nil {
		return nil, err
	}
	return unsafe.Slice((*byte)(p), size), nil
}

// HostFree releases a slice from HostAlloc.
func HostFree(b []byte) error {
	if cap(b) == 0 {
		return nil
	}
	return toError(C.cfsec_host_free(unsafe.Pointer(unsafe.SliceData(b[:1]))))
}

func (e *Engine) Verify(shards [][]byte) (bool, error) {
	v := newShardVec(shards)
	defer v.free()
	var ok C.int
	err := toError(C.cfsec_rs_verify(e.h, v.ptr(), C.int(v.n), C.CFSEC_MEM_HOST, nil, &ok))
	return ok != 0, err
}

// prepareMissing gives every zero-length shard a buffer of the shard size, as
// KRS/reedsolomon.go:1514-1518 does (reuse cap, else a 64-byte aligned allocation).
func prepareMissing(shards [][]byte) {
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

func (e *Engine) Reconstruct(shards [][]byte) error {
	prepareMissing(shards)
	v := newShardVec(shards)
	defer v.free()
	st := C.cfsec_rs_reconstruct(e.h, v.ptr(), C.int(v.n), C.CFSEC_MEM_HOST, nil)
	v.lens(shards)
	return toError(st)
}

func (e *Engine) ReconstructData(shards [][]byte) error {
	prepareMissing(shards)
	v := newShardVec(shards)
	defer v.free()
	st := C.cfsec_rs_reconstruct_data(e.h, v.ptr(), C.int(v.n), C.CFSEC_MEM_HOST, nil)
	v.lens(shards)
	return toError(st)
}

func (e *Engine) Split(data []byte) ([][]byte, error) {
	total := e.dataShards + e.parityShards
	if len(data) == 0 {
		return nil, reedsolomon.ErrShortData
	}
	out := make([]C.cfsec_shard, total)
	var pin runtime.Pinner
	defer pin.Unpin()
	base := &data[:cap(data)][0]
	pin.Pin(base)
	var need C.size_t
	st := C.cfsec_rs_split(e.h, (*C.uint8_t)(unsafe.Pointer(base)), C.size_t(len(data)), C.size_t(cap(data)),
		&out[0], nil, 0, &need)
	var pad []byte
	if st == C.CFSEC_ERR_INVALID_ARG && need > 0 {
		pad = reedsolomon.AllocAligned(1, int(need))[0]
		pin.Pin(&pad[0])
		st = C.cfsec_rs_split(e.h, (*C.uint8_t)(unsafe.Pointer(base)), C.size_t(len(data)), C.size_t(cap(data)),
			&out[0], (*C.uint8_t)(unsafe.Pointer(&pad[0])), need, &need)
	}
	if err := toError(st); err != nil {
		return nil, err
	}
	full := data[:cap(data)]
	res := make([][]byte, total)
	for i, s := range out {
		off := uintptr(unsafe.Pointer(s.data)) - uintptr(unsafe.Pointer(base))
		if off < uintptr(len(full)) {
			res[i] = full[off : off+uintptr(s.len) : off+uintptr(s.len)]
		} else {
			off = uintptr(unsafe.Pointer(s.data)) - uintptr(unsafe.Pointer(&pad[0]))
			res[i] = pad[off : off+uintptr(s.len) : off+uintptr(s.len)]
		}
	}
	return res, nil
}

// Join is pure host bookkeeping (KRS/reedsolomon.go:1646-1684); it stays in Go so the
// io.Writer sees exactly the reference's write pattern.
func (e *Engine) Join(dst io.Writer, shards [][]byte, outSize int) error {
	if len(shards) < e.dataShards {
		return reedsolomon.ErrTooFewShards
	}
	shards = shards[:e.dataShards]
	size := 0
	for _, shard := range shards {
		if shard == nil {
			return reedsolomon.ErrReconstructRequired
		}
		size += len(shard)
		if size >= outSize {
			break
		}
	}
	if size < outSize {
		return reedsolomon.ErrShortData
	}
	write := outSize
	for _, shard := range shards {
		if write < len(shard) {
			_, err := dst.Write(shard[:write])
			return err
		}
		n, err := dst.Write(shard)
		if err != nil {
			return err
		}
		write -= n
	}
	return nil
}

func (e *Engine) EncodeIdx(dataShard []byte, idx int, parity [][]byte) error {
	return reedsolomon.ErrNotSupported
}

func (e *Engine) ReconstructSome(shards [][]byte, required []bool) error {
	return reedsolomon.ErrNotSupported
}

func (e *Engine) Update(shards [][]byte, newDatashards [][]byte) error {
	return reedsolomon.ErrNotSupported
}

// ---- crc32block framing (blobstore/common/crc32block) ----

// ErrMismatchedCrc / ErrInvalidBlock mirror crc32block's sentinels (common/crc32block/util.go:29-30);
// a shim dropped into crc32block returns that package's own values instead.
var (
	ErrMismatchedCrc = errors.New("crc32block: mismatched checksum")
	ErrInvalidBlock  = errors.New("crc32block: invalid block buffer")
)

// BlockEncode frames payload in blockLen-byte crc32block blocks (crc32block.Encoder.Encode,
// encode.go:48-58) on the GPU and returns the framed bytes together with crc32.ChecksumIEEE of the
// whole payload -- the shard checksum blobnode's datafile.Write takes on the way
// (core/storage/datafile.go:345-373) -- from the same single pass.
func BlockEncode(payload []byte, blockLen int64) ([]byte, uint32, error) {
	total := int64(C.cfsec_crc32block_encode_size(C.int64_t(len(payload)), C.int64_t(blockLen)))
	if total < 0 {
		return nil, 0, ErrInvalidBlock
	}
	out := make([]byte, total)
	if len(payload) == 0 {
		return out, 0, nil
	}
	var pin runtime.Pinner
	pin.Pin(&payload[0])
	pin.Pin(&out[0])
	defer pin.Unpin()
	var crc C.uint32_t
	st := C.cfsec_crc32block_encode((*C.uint8_t)(unsafe.Pointer(&payload[0])), C.int64_t(len(payload)),
		C.int64_t(blockLen), (*C.uint8_t)(unsafe.Pointer(&out[0])), &crc, C.CFSEC_MEM_HOST, -1, nil)
	if st == C.CFSEC_ERR_INVALID_BLOCK {
		return nil, 0, ErrInvalidBlock
	}
	return out, uint32(crc), toError(st)
}

// BlockDecode returns payload bytes [from, to) of a framed object whose payload is size bytes,
// checking every block the range touches (crc32block.Decoder.Reader, decode.go:122-146).
func BlockDecode(framed []byte, size, from, to, blockLen int64) ([]byte, error) {
	if from < 0 || from > to || to > size {
		return nil, errInvalidArg
	}
	out := make([]byte, to-from)
	var pin runtime.Pinner
	defer pin.Unpin()
	var src, dst *C.uint8_t
	if len(framed) > 0 {
		pin.Pin(&framed[0])
		src = (*C.uint8_t)(unsafe.Pointer(&framed[0]))
	}
	if len(out) > 0 {
		pin.Pin(&out[0])
		dst = (*C.uint8_t)(unsafe.Pointer(&out[0]))
	}
	var bad C.int64_t
	switch st := C.cfsec_crc32block_decode(src, C.int64_t(len(framed)), C.int64_t(size), C.int64_t(blockLen),
		C.int64_t(from), C.int64_t(to), dst, &bad, C.CFSEC_MEM_HOST, -1, nil); st {
	case C.CFSEC_ERR_MISMATCHED_CRC:
		return nil, ErrMismatchedCrc
	case C.CFSEC_ERR_INVALID_BLOCK:
		return nil, ErrInvalidBlock
	case C.CFSEC_ERR_SHORT_DATA:
		// the framed object ends before the blocks the range touches: what the reference's
		// SectionReader reports (decode.go:94-97, 126-130)
		return nil, io.ErrUnexpectedEOF
	default:
		return out, toError(st)
	}
}
