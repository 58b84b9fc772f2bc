"""Marshalling of Python shard lists into cfsec_shard arrays and back.

A Go [][]byte becomes a Python list whose entries are 1-D uint8 buffers:
numpy arrays (host memory, CFSEC_MEM_HOST) or torch uint8 tensors on a HIP
device (CFSEC_MEM_DEVICE).  len(entry) == 0 or None marks a missing shard,
as in KRS/reedsolomon.go:1416-1428.  Python buffers carry no Go capacity, so a
missing entry is given a fresh zeroed buffer of the shard size before the call
(what KRS does with AllocAligned when cap is short, reedsolomon.go:1514-1518,
and ec.fillFullShards with make, encoder.go:199-210); after the call each
list entry is re-sliced to the length the engine reported.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


def _nbytes(x) -> int:
    if x is None:
        return 0
    if _is_torch(x):
        return x.numel() * x.element_size()
    return int(x.size)


def _ptr(x) -> int:
    if _is_torch(x):
        return x.data_ptr()
    return x.ctypes.data


class Marshal:
    def __init__(self, shards, fill_size=None):
        self.shards = shards
        self.n = len(shards)
        self.mem = None
        self.like = None
        for s in shards:
            if s is not None and _nbytes(s) > 0:
                kind = _lib.MEM_DEVICE if _is_torch(s) else _lib.MEM_HOST
                if _is_torch(s) and not s.is_cuda:
                    raise TypeError("torch shards must live on a HIP device")
                if self.mem is None:
                    self.mem, self.like = kind, s
                elif self.mem != kind:
                    raise TypeError("mixing host and device shards in one call")
        if self.mem is None:
            self.mem = _lib.MEM_HOST
        self.arr = (_lib.Shard * max(self.n, 1))()
        self.orig_len = []
        self.alloc = {}
        for i, s in enumerate(shards):
            ln = _nbytes(s)
            if s is not None and not _is_torch(s):
                if s.dtype != np.uint8 or s.ndim != 1 or not s.flags.c_contiguous:
                    raise TypeError("host shards must be 1-D contiguous uint8 numpy arrays")
            if s is not None and _is_torch(s):
                import torch
                if s.dtype != torch.uint8 or s.dim() != 1 or not s.is_contiguous():
                    raise TypeError("device shards must be 1-D contiguous uint8 tensors")
            self.orig_len.append(ln)
            if ln == 0 and fill_size:
                buf = self._new(fill_size)
                self.alloc[i] = buf
                self.arr[i] = _lib.Shard(_ptr(buf), 0, fill_size)
            elif ln == 0:
                self.arr[i] = _lib.Shard(None, 0, 0)
            else:
                self.arr[i] = _lib.Shard(_ptr(s), ln, ln)

    def _new(self, size):
        if self.mem == _lib.MEM_DEVICE:
            import torch
            return torch.zeros(size, dtype=torch.uint8, device=self.like.device)
        return np.zeros(size, np.uint8)

    def ptr(self):
        return self.arr

    def writeback(self):
        """Re-slice every entry to the length the engine left in its header."""
        for i in range(self.n):
            ln = self.arr[i].len
            if ln == self.orig_len[i]:
                continue
            base = self.alloc.get(i)
            if base is None:
                base = self.shards[i]
            if base is None:
                continue
            self.shards[i] = base[:ln]


def shard_size(shards) -> int:
    for s in shards:
        ln = _nbytes(s)
        if ln:
            return ln
    return 0


def stream_ptr(stream, like=None, device=None):
    """The hipStream_t to pass for `stream`.  None means the caller's current PyTorch stream on the
    device the call runs on (the device of the torch buffer `like`, else `device`): a call must be
    ordered after the kernel that produced its input, and PyTorch's side streams are non-blocking,
    so the C ABI's NULL (ordered after the legacy default stream only) would race with them."""
    if stream is None:
        import sys
        torch = sys.modules.get("torch")
        if torch is None:
            return None
        if like is not None and _is_torch(like) and like.is_cuda:
            dev = like.device
        elif device is not None and device >= 0:
            dev = torch.device("cuda", device)
        else:
            return None
        if not torch.cuda.is_initialized():
            return None  # nothing can be queued on a stream yet
        return torch.cuda.current_stream(dev).cuda_stream or None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream  # torch.cuda.Stream


def ptr_array(ptrs):
    """A ctypes array of device pointers; an existing ctypes array passes through (callers
    that launch the same batch repeatedly build it once)."""
    if isinstance(ptrs, ctypes.Array):
        return ptrs
    return (ctypes.c_void_p * len(ptrs))(*[int(p) for p in ptrs])


class BatchMarshal:
    """A list of stripes (each a list of shards, as Marshal takes) as one cfsec_shard array of
    nstripes * n entries, stripe-major; missing shards get fresh buffers of their stripe's size."""

    def __init__(self, stripes, n, fill=False):
        self.parts = []
        self.n = n
        self.mem = None
        for st in stripes:
            if len(st) != n:
                raise ValueError(f"every stripe needs {n} shards")
            m = Marshal(st, fill_size=shard_size(st) if fill else None)
            if self.mem is None:
                self.mem = m.mem
            elif m.mem != self.mem and any(_nbytes(x) for x in st):
                raise TypeError("mixing host and device stripes in one batch")
            self.parts.append(m)
        if self.mem is None:
            self.mem = _lib.MEM_HOST
        self.arr = (_lib.Shard * max(len(stripes) * n, 1))()
        for s, m in enumerate(self.parts):
            for i in range(n):
                self.arr[s * n + i] = m.arr[i]

    def writeback(self):
        for s, m in enumerate(self.parts):
            for i in range(self.n):
                m.arr[i] = self.arr[s * self.n + i]
            m.writeback()
