//go:build !go1.21

package cfsec

/*
#include <stdlib.h>
#include "cfsec.h"
*/
import "C"

import "unsafe"

// callVec for Go releases without runtime.Pinner (CubeFS's Go 1.17): a shard vector that is not one
// contiguous stripe is staged through C memory -- the C array then holds C pointers only, which
// cgo allows on every release.  Each shard's slot holds its bytes up to the shard size, a missing
// shard's spare capacity included (fillFullShards reuses it, encoder.go:199-210); afterwards every
// shard is copied back and re-sliced to the length fn left in its header.  Costs two host copies;
// ec.Buffer stripes never come here (stripeOf sends them through the contiguous entry points).
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
	off := make([]int, n+1)
	for i, s := range shards {
		sz := len(s)
		if sz < size && cap(s) >= size {
			sz = size
		}
		off[i+1] = off[i] + sz
	}
	buf := C.malloc(C.size_t(off[n] + 1))
	defer C.free(buf)
	mem := unsafe.Slice((*byte)(buf), off[n]+1)
	arr := (*C.cfsec_shard)(C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(C.cfsec_shard{}))))
	defer C.free(unsafe.Pointer(arr))
	elems := unsafe.Slice(arr, n)
	for i, s := range shards {
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
