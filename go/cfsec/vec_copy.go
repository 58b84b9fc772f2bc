//go:build !go1.21

package cfsec

/*
#include <stdlib.h>
#include "cfsec.h"
*/
import "C"

import "unsafe"

// callVec for Go releases without runtime.Pinner (CubeFS's Go 1.17).  A shard in HostAlloc memory
// (C memory, regions.go) goes into the C array as it is.  A shard in Go memory is staged through C
// memory -- the C array then holds C pointers only, which cgo allows on every release: its slot
// holds its bytes up to the shard size, a missing shard's spare capacity included (fillFullShards
// reuses it, encoder.go:199-210), and afterwards it is copied back.  Every shard is re-sliced to the
// length fn left in its header.  A tasklet whose shard buffers come from HostAlloc (blobnode's
// ShardsBuf, INTEGRATION.md §3a) costs no host copy; registered ec.Buffer stripes never come here
// (stripeOf sends them through the contiguous entry points).
func callVec(shards [][]byte, fn func(*C.cfsec_shard, C.int) C.int) C.int {
	n := len(shards)
	if n == 0 {
		return fn(nil, 0)
	}
	size := 0
	for _, s := range shards {
		if len(s) != 0 {
			size = len(s)
			break
		}
	}
	direct := make([]bool, n)
	off := make([]int, n+1)
	for i, s := range shards {
		direct[i] = inCMem(s)
		sz := 0
		if !direct[i] {
			sz = len(s)
			if sz < size && cap(s) >= size {
				sz = size
			}
		}
		off[i+1] = off[i] + sz
	}
	var mem []byte
	if off[n] > 0 {
		buf := C.malloc(C.size_t(off[n]))
		defer C.free(buf)
		mem = unsafe.Slice((*byte)(buf), off[n])
	}
	arr := (*C.cfsec_shard)(C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(C.cfsec_shard{}))))
	defer C.free(unsafe.Pointer(arr))
	elems := unsafe.Slice(arr, n)
	for i, s := range shards {
		if direct[i] {
			elems[i] = C.cfsec_shard{data: (*C.uint8_t)(unsafe.Pointer(&s[:1][0])), len: C.size_t(len(s)),
				cap: C.size_t(cap(s))}
			continue
		}
		slot := mem[off[i]:off[i+1]]
		copy(slot, s[:cap(s)])
		elems[i] = C.cfsec_shard{data: nil, len: C.size_t(len(s)), cap: C.size_t(len(slot))}
		if len(slot) > 0 {
			elems[i].data = (*C.uint8_t)(unsafe.Pointer(&slot[0]))
		}
	}
	st := fn(arr, C.int(n))
	for i, el := range elems {
		l := int(el.len)
		if direct[i] {
			shards[i] = shards[i][:l] // rebuilt in place, l <= cap
			continue
		}
		dst := shards[i]
		if l > cap(dst) {
			dst = make([]byte, l)
		}
		dst = dst[:l]
		copy(dst, mem[off[i]:off[i]+l])
		shards[i] = dst
	}
	return st
}
