package cfsec

import (
	"sort"
	"sync"
	"unsafe"
)

// Allocation regions the binding may address as a whole.
//
// cgo's pointer rules (Go 1.6 onward) let C receive a Go pointer to memory that holds no Go pointers,
// and C may then reach the whole allocation that pointer points into -- but nothing beyond it.  A
// shard vector whose shards merely sit at one stride (stripeOf) is one allocation only when the
// caller knows it is: ec.Buffer carves every shard of a stripe from one []byte (common/ec/buf.go:
// 83-84), but separately allocated equal-size buffers from one size-class span can line up the same
// way.  So the one-pointer (contiguous) entry points are used only for stripes that lie inside a
// region registered here:
//
//   - RegisterBuffer(buf): the caller vouches that buf is one allocation (ec.Buffer's ECDataBuf,
//     blobnode's per-vuid shard buffers); the registry keeps buf alive until UnregisterBuffer;
//   - HostAlloc registers its page-locked C memory itself (HostFree removes it).  C memory is not Go
//     memory, so shards in it may also sit in a C array on every Go release: callVec passes them
//     without staging or pinning (vec_copy.go, vec_pin.go).
type region struct {
	base, end uintptr // [base, end)
	cmem      bool    // C memory from HostAlloc
	keep      []byte  // Go memory: referenced while registered
}

var (
	regMu   sync.RWMutex
	regions []region // sorted by base, disjoint
)

func addRegion(b []byte, cmem bool) {
	if cap(b) == 0 {
		return
	}
	base := uintptr(unsafe.Pointer(&b[:1][0]))
	r := region{base: base, end: base + uintptr(cap(b)), cmem: cmem}
	if !cmem {
		r.keep = b[:cap(b)]
	}
	regMu.Lock()
	defer regMu.Unlock()
	i := sort.Search(len(regions), func(i int) bool { return regions[i].base >= base })
	if i < len(regions) && regions[i].base == base {
		regions[i] = r
		return
	}
	regions = append(regions, region{})
	copy(regions[i+1:], regions[i:])
	regions[i] = r
}

func removeRegion(b []byte) {
	if cap(b) == 0 {
		return
	}
	base := uintptr(unsafe.Pointer(&b[:1][0]))
	regMu.Lock()
	defer regMu.Unlock()
	i := sort.Search(len(regions), func(i int) bool { return regions[i].base >= base })
	if i < len(regions) && regions[i].base == base {
		regions = append(regions[:i], regions[i+1:]...)
	}
}

// regionOf returns the registered region holding [p, p+n), if any.
func regionOf(p uintptr, n int) (region, bool) {
	regMu.RLock()
	defer regMu.RUnlock()
	i := sort.Search(len(regions), func(i int) bool { return regions[i].base > p }) - 1
	if i < 0 {
		return region{}, false
	}
	r := regions[i]
	if p >= r.base && p+uintptr(n) <= r.end {
		return r, true
	}
	return region{}, false
}

// inCMem reports whether s's whole capacity lies in HostAlloc memory.
func inCMem(s []byte) bool {
	if cap(s) == 0 {
		return false
	}
	r, ok := regionOf(uintptr(unsafe.Pointer(&s[:1][0])), cap(s))
	return ok && r.cmem
}

// RegisterBuffer declares buf (its whole capacity) one allocation whose stripes -- shards carved at
// one stride from it, as ec.Buffer and Split do -- may cross the C ABI as a single pointer.  Call it
// where the buffer is created (ec.NewBuffer's ECDataBuf, blobnode's shard buffers) and
// UnregisterBuffer before the buffer is returned to its pool.  Unregistered stripes still work; they
// take the shard-vector path.
func RegisterBuffer(buf []byte) { addRegion(buf, false) }

// UnregisterBuffer removes a buffer registered with RegisterBuffer.
func UnregisterBuffer(buf []byte) { removeRegion(buf) }
