// Package cfsec is the cgo binding a CubeFS maintainer drops into
// blobstore/common/ec to run the EC engine on MI355X GPUs.
//
// It implements github.com/klauspost/reedsolomon.Encoder (the seam that
// blobstore/common/ec/encoder.go:86 and :95 construct) over the C ABI in
// include/cfsec.h.  The methods CubeFS calls go to libcfsec.so -- Encode, Verify, Reconstruct,
// ReconstructData -- or, for Split and Join (host bookkeeping, no coding), stay in Go as the
// reference writes them; EncodeIdx, ReconstructSome and Update, which CubeFS never calls, return
// reedsolomon.ErrNotSupported.
//
// Go releases.  CubeFS builds with Go 1.17 (go.mod:3, docker/Dockerfile:1), whose cgo rules forbid a
// C array holding Go pointers.  So every call first looks for the one-allocation layout that
// ec.Buffer and Split produce (stripeOf: shard i at base + i*stride, inside one buffer registered
// with RegisterBuffer or allocated by HostAlloc) and passes that stripe as a single pointer to the
// cfsec_*_contig entry points -- legal on every Go release.  Any other shard vector goes through
// callVec: shards in HostAlloc memory are C memory and go into the C array as they are; Go memory is
// pinned with Go >= 1.21 (runtime.Pinner, vec_pin.go) and staged through C memory before that
// (vec_copy.go).
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
	"sync/atomic"
	"unsafe"

	"github.com/klauspost/reedsolomon"
)

// stripeOf reports whether every shard is size bytes at one stride from the first (ec.Buffer's
// layout, common/ec/buf.go:83-84, which encoder.Split carves) inside one registered allocation
// (regions.go: RegisterBuffer, HostAlloc): then the stripe crosses the C ABI as its base pointer
// alone (cfsec_*_contig).  Shards that only happen to sit at one stride are not enough -- cgo lets C
// reach the allocation a pointer points into, nothing beyond it.
func stripeOf(shards [][]byte) (base *C.uint8_t, size, stride int, ok bool) {
	if len(shards) == 0 || len(shards[0]) == 0 {
		return nil, 0, 0, false
	}
	size = len(shards[0])
	p0 := uintptr(unsafe.Pointer(&shards[0][0]))
	stride = size
	if len(shards) > 1 && len(shards[1]) == size {
		stride = int(uintptr(unsafe.Pointer(&shards[1][0])) - p0)
	}
	if stride < size {
		return nil, 0, 0, false
	}
	for i, s := range shards {
		if len(s) != size || uintptr(unsafe.Pointer(&s[0])) != p0+uintptr(i*stride) {
			return nil, 0, 0, false
		}
	}
	if _, one := regionOf(p0, (len(shards)-1)*stride+size); !one {
		// an equal-stride stripe outside every registered allocation (an ec.Buffer nobody passed
		// to RegisterBuffer): it still works, through callVec -- on Go < 1.21 that stages every
		// shard through C memory, two host copies per call.  Counted, so an integration that
		// forgot RegisterBuffer sees it (UnregisteredStripes).
		atomic.AddUint64(&unregisteredStripes, 1)
		return nil, 0, 0, false
	}
	return (*C.uint8_t)(unsafe.Pointer(&shards[0][0])), size, stride, true
}

var unregisteredStripes uint64

// UnregisteredStripes is the number of calls so far whose shards formed one equal-stride stripe
// (ec.Buffer's layout) that lay in no RegisterBuffer / HostAlloc region, so it missed the single-
// pointer zero-copy path.  Nonzero means some ec.Buffer allocation should be registered.
func UnregisteredStripes() uint64 { return atomic.LoadUint64(&unregisteredStripes) }

// stripeOfMissing is stripeOf for a Reconstruct input: a missing shard (len 0) counts when its
// capacity holds the shard at its place in the stripe; missing lists those indices.
func stripeOfMissing(shards [][]byte) (base *C.uint8_t, size, stride int, missing []C.int, ok bool) {
	first := -1
	for i, s := range shards {
		if len(s) != 0 {
			first, size = i, len(s)
			break
		}
	}
	if first < 0 {
		return nil, 0, 0, nil, false
	}
	addr := make([]uintptr, len(shards))
	for i, s := range shards {
		switch {
		case len(s) == size:
			addr[i] = uintptr(unsafe.Pointer(&s[0]))
		case len(s) == 0 && cap(s) >= size:
			addr[i] = uintptr(unsafe.Pointer(&s[:1][0]))
			missing = append(missing, C.int(i))
		default:
			return nil, 0, 0, nil, false
		}
	}
	stride = size
	if len(shards) > 1 {
		stride = int(addr[1] - addr[0])
	}
	if stride < size {
		return nil, 0, 0, nil, false
	}
	for i := range shards {
		if addr[i] != addr[0]+uintptr(i*stride) {
			return nil, 0, 0, nil, false
		}
	}
	if _, one := regionOf(addr[0], (len(shards)-1)*stride+size); !one {
		return nil, 0, 0, nil, false
	}
	return (*C.uint8_t)(unsafe.Pointer(addr[0])), size, stride, missing, true
}

func cints(v []int) ([]C.int, *C.int) {
	if len(v) == 0 {
		return nil, nil
	}
	c := make([]C.int, len(v))
	for i, x := range v {
		c[i] = C.int(x)
	}
	return c, &c[0]
}

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

func (e *Engine) Encode(shards [][]byte) error {
	if base, size, stride, ok := stripeOf(shards); ok {
		return toError(C.cfsec_rs_encode_contig(e.h, base, C.size_t(size), C.size_t(stride), C.int(len(shards)),
			C.CFSEC_MEM_HOST, nil))
	}
	return toError(callVec(shards, func(v *C.cfsec_shard, n C.int) C.int {
		return C.cfsec_rs_encode(e.h, v, n, C.CFSEC_MEM_HOST, nil)
	}))
}

// EncodeCRC is Encode followed by crc32.ChecksumIEEE of every shard -- what access computes
// right after encoding (blobstore/access/stream_put.go:249-253) -- in one fused GPU pass.
func (e *Engine) EncodeCRC(shards [][]byte) ([]uint32, error) {
	crcs := make([]uint32, len(shards)+1) // +1: a valid address even for an empty vector
	st := callVec(shards, func(v *C.cfsec_shard, n C.int) C.int {
		return C.cfsec_rs_encode_crc(e.h, v, n, C.CFSEC_MEM_HOST, nil, (*C.uint32_t)(unsafe.Pointer(&crcs[0])))
	})
	return crcs[:len(shards)], toError(st)
}

// HostAlloc returns size bytes of page-locked C memory (cfsec_host_alloc) as a byte slice: the
// allocation hook for resourcepool.NewMemPoolWith (common/resourcepool/mempool.go:60), so
// ec.Buffer shards are coded in place over PCIe, and for blobnode's shard buffers
// (blobnode/base/workutils/buf_pool.go:26-29).  The block is registered as one region (regions.go):
// its stripes take the one-pointer entry points and its shards sit in C arrays without staging or
// pinning on every Go release.  Release it with HostFree.
func HostAlloc(size int) ([]byte, error) {
	if size <= 0 {
		return nil, nil
	}
	var p unsafe.Pointer
	if err := toError(C.cfsec_host_alloc(C.size_t(size), &p)); err != nil {
		return nil, err
	}
	b := unsafe.Slice((*byte)(p), size)
	addRegion(b, true)
	return b, nil
}

// HostFree releases a slice from HostAlloc.
func HostFree(b []byte) error {
	if cap(b) == 0 {
		return nil
	}
	removeRegion(b)
	return toError(C.cfsec_host_free(unsafe.Pointer(&b[:1][0])))
}

func (e *Engine) Verify(shards [][]byte) (bool, error) {
	ok := make([]C.int, 1)
	if base, size, stride, contig := stripeOf(shards); contig {
		err := toError(C.cfsec_rs_verify_contig(e.h, base, C.size_t(size), C.size_t(stride), C.int(len(shards)),
			C.CFSEC_MEM_HOST, nil, &ok[0]))
		return ok[0] != 0, err
	}
	err := toError(callVec(shards, func(v *C.cfsec_shard, n C.int) C.int {
		return C.cfsec_rs_verify(e.h, v, n, C.CFSEC_MEM_HOST, nil, &ok[0])
	}))
	return ok[0] != 0, err
}

// prepareMissing gives the shards KRS's reconstruct rebuilds a buffer of the shard size when their
// capacity is short, as KRS/reedsolomon.go:1514-1518 and :1539-1543 do (reuse cap, else a 64-byte
// aligned allocation) -- and only those: nothing when the stripe is complete (or, for
// ReconstructData, its data is), nothing when too few shards are present (ErrTooFewShards comes
// first, :1418-1441), and no parity shard for ReconstructData.  The C side writes into cap only.
func prepareMissing(shards [][]byte, dataShards int, dataOnly bool) {
	size, present, dataPresent := 0, 0, 0
	for i, s := range shards {
		if len(s) != 0 {
			if size == 0 {
				size = len(s)
			}
			present++
			if i < dataShards {
				dataPresent++
			}
		}
	}
	if size == 0 || present == len(shards) || present < dataShards || (dataOnly && dataPresent == dataShards) {
		return
	}
	for i, s := range shards {
		if dataOnly && i >= dataShards {
			break
		}
		if len(s) == 0 && cap(s) < size {
			shards[i] = reedsolomon.AllocAligned(1, size)[0][:0]
		}
	}
}

func (e *Engine) reconstruct(shards [][]byte, dataOnly bool) error {
	donly := C.int(0)
	if dataOnly {
		donly = 1
	}
	// ec.Buffer's stripe with some shards marked missing: one pointer, rebuilt in place
	if base, size, stride, missing, ok := stripeOfMissing(shards); ok && len(shards) == e.dataShards+e.parityShards {
		var mp *C.int
		if len(missing) > 0 {
			mp = &missing[0]
		}
		err := toError(C.cfsec_rs_reconstruct_contig(e.h, base, C.size_t(size), C.size_t(stride), C.int(len(shards)),
			mp, C.int(len(missing)), donly, C.CFSEC_MEM_HOST, nil))
		if err == nil {
			// the rebuilt shards get their length, as KRS/reedsolomon.go:1514-1518 and :1539-1543 do
			present := len(shards) - len(missing)
			dataPresent := 0
			for i := 0; i < e.dataShards; i++ {
				if len(shards[i]) != 0 {
					dataPresent++
				}
			}
			if present < len(shards) && !(dataOnly && dataPresent == e.dataShards) {
				for _, i := range missing {
					if !dataOnly || int(i) < e.dataShards {
						shards[i] = shards[i][:size]
					}
				}
			}
		}
		return err
	}
	prepareMissing(shards, e.dataShards, dataOnly)
	return toError(callVec(shards, func(v *C.cfsec_shard, n C.int) C.int {
		if dataOnly {
			return C.cfsec_rs_reconstruct_data(e.h, v, n, C.CFSEC_MEM_HOST, nil)
		}
		return C.cfsec_rs_reconstruct(e.h, v, n, C.CFSEC_MEM_HOST, nil)
	}))
}

func (e *Engine) Reconstruct(shards [][]byte) error { return e.reconstruct(shards, false) }

func (e *Engine) ReconstructData(shards [][]byte) error { return e.reconstruct(shards, true) }

// Split and Join are host bookkeeping -- slice headers, a zero fill, one copy of the partial tail --
// with no coding arithmetic, so the shim keeps them in Go (KRS/reedsolomon.go:1574-1684) rather
// than sending Go memory through C: the C ABI's cfsec_rs_split / cfsec_rs_join run the same
// algorithm for C callers (pinned by tests/test_capi.py), but a C function that writes addresses of
// Go buffers into an array outlives the cgo call's pointer rules, and a Join through C costs two
// copies of the object where the reference writes the shard slices straight to dst.

// Split: the data shards are views of data itself (its spare capacity zeroed and used), the shards
// past the end of data come from AllocAligned (64-byte aligned, stride and capacity rounded up to
// 64), the bytes after the last full shard copied into them in order.
func (e *Engine) Split(data []byte) ([][]byte, error) {
	n := len(data)
	if n == 0 {
		return nil, reedsolomon.ErrShortData
	}
	tot := e.dataShards + e.parityShards
	if tot == 1 {
		return [][]byte{data}, nil
	}
	per := (n + e.dataShards - 1) / e.dataShards
	// usable bytes of data: its length, or its capacity up to tot*per (zeroed past the length)
	usable := n
	if c := cap(data); c > n {
		usable = tot * per
		if c < usable {
			usable = c
		}
		tail := data[n:usable]
		for i := range tail {
			tail[i] = 0
		}
	}
	buf := data[:usable]
	inPlace := usable / per
	if inPlace > tot {
		inPlace = tot
	}
	out := make([][]byte, tot)
	for i := 0; i < inPlace; i++ {
		out[i] = buf[i*per : (i+1)*per : (i+1)*per]
	}
	if inPlace < tot {
		pad := reedsolomon.AllocAligned(tot-inPlace, per)
		var rest []byte
		if inPlace*per < n {
			rest = data[inPlace*per : n]
		}
		for j := range pad {
			rest = rest[copy(pad[j], rest):]
			out[inPlace+j] = pad[j]
		}
	}
	return out, nil
}

// Join: ErrTooFewShards, ErrReconstructRequired (a nil data shard before outSize bytes are covered)
// and ErrShortData are decided before anything is written or allocated; then one Write per data
// shard, the last cut at outSize.
func (e *Engine) Join(dst io.Writer, shards [][]byte, outSize int) error {
	if len(shards) < e.dataShards {
		return reedsolomon.ErrTooFewShards
	}
	data := shards[:e.dataShards]
	have := 0
	for _, s := range data {
		if s == nil {
			return reedsolomon.ErrReconstructRequired
		}
		if have += len(s); have >= outSize {
			break
		}
	}
	if have < outSize {
		return reedsolomon.ErrShortData
	}
	left := outSize
	for _, s := range data {
		if left < len(s) {
			_, err := dst.Write(s[:left])
			return err
		}
		w, err := dst.Write(s)
		if err != nil {
			return err
		}
		left -= w
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
	crc := make([]C.uint32_t, 1)
	// Go pointers passed as arguments to memory holding no Go pointers: legal without pinning
	st := C.cfsec_crc32block_encode((*C.uint8_t)(unsafe.Pointer(&payload[0])), C.int64_t(len(payload)),
		C.int64_t(blockLen), (*C.uint8_t)(unsafe.Pointer(&out[0])), &crc[0], C.CFSEC_MEM_HOST, -1, nil)
	if st == C.CFSEC_ERR_INVALID_BLOCK {
		return nil, 0, ErrInvalidBlock
	}
	return out, uint32(crc[0]), toError(st)
}

// BlockDecode returns payload bytes [from, to) of a framed object whose payload is size bytes,
// checking every block the range touches (crc32block.Decoder.Reader, decode.go:122-146).
func BlockDecode(framed []byte, size, from, to, blockLen int64) ([]byte, error) {
	if from < 0 || from > to || to > size {
		return nil, errInvalidArg
	}
	out := make([]byte, to-from)
	var src, dst *C.uint8_t
	if len(framed) > 0 {
		src = (*C.uint8_t)(unsafe.Pointer(&framed[0]))
	}
	if len(out) > 0 {
		dst = (*C.uint8_t)(unsafe.Pointer(&out[0]))
	}
	bad := make([]C.int64_t, 1)
	switch st := C.cfsec_crc32block_decode(src, C.int64_t(len(framed)), C.int64_t(size), C.int64_t(blockLen),
		C.int64_t(from), C.int64_t(to), dst, &bad[0], C.CFSEC_MEM_HOST, -1, nil); st {
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
