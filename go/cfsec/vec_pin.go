//go:build go1.21

package cfsec

/*
#include <stdlib.h>
#include "cfsec.h"
*/
import "C"

import (
	"runtime"
	"unsafe"
)

// callVec hands a shard vector that is not one contiguous stripe to fn as a C array of
// {data, len, cap} pointing at the caller's own buffers, pinned for the call (runtime.Pinner, Go
// >= 1.21: pinned Go pointers may sit in C memory), then re-slices each shard to the length fn left
// in its header (Reconstruct's rebuilt shards, fillFullShards).  The C side keeps no pointer after
// the call.
func callVec(shards [][]byte, fn func(*C.cfsec_shard, C.int) C.int) C.int {
	n := len(shards)
	if n == 0 {
		return fn(nil, 0)
	}
	var pin runtime.Pinner
	defer pin.Unpin()
	arr := (*C.cfsec_shard)(C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(C.cfsec_shard{}))))
	defer C.free(unsafe.Pointer(arr))
	elems := unsafe.Slice(arr, n)
	for i, s := range shards {
		elems[i] = C.cfsec_shard{data: nil, len: C.size_t(len(s)), cap: C.size_t(cap(s))}
		if cap(s) > 0 {
			p := &s[:cap(s)][0]
			if !inCMem(s) { // HostAlloc memory is C memory: nothing to pin
				pin.Pin(p)
			}
			elems[i].data = (*C.uint8_t)(unsafe.Pointer(p))
		}
	}
	st := fn(arr, C.int(n))
	for i, el := range elems {
		if int(el.len) != len(shards[i]) {
			shards[i] = shards[i][:int(el.len)]
		}
	}
	return st
}
