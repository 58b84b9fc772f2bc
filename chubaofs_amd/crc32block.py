"""crc32block -- mirror of blobstore/common/crc32block backed by libcfsec.so's gfx950 framing
kernel (cfsec_crc32block_*).

A framed object is a run of blocks of `block_len` bytes, each the little-endian
crc32.ChecksumIEEE of its payload followed by the payload (block.go:34-49, encode.go:87-109).

    framed, crc = Encode(payload)              # Encoder.Encode; crc = the whole shard's
                                               # ChecksumIEEE that blobnode takes on the way
                                               # (core/storage/datafile.go:345-373)
    part = Decode(framed, size, from_, to)     # Decoder.Reader(from, to) read to the end
                                               # (decode.go:122-146, datafile.go:406-426)

Buffers are 1-D uint8 numpy arrays (host memory; arrays from _lib.pinned_empty are read and
written in place) or uint8 torch tensors on a HIP device.  Errors are the Go sentinels:
ErrInvalidBlock (block length not a positive multiple of 4096), ErrMismatchedCrc.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._shards import _is_torch, _nbytes, _ptr, ptr_array, stream_ptr

DefaultBlockSize = 64 * 1024  # defaultCrc32BlockSize, block.go:22-24


def EncodeSize(size: int, blockLen: int = DefaultBlockSize) -> int:
    """util.go:50-57 (panics with ErrInvalidBlock there; raises here)."""
    v = _lib.lib().cfsec_crc32block_encode_size(int(size), int(blockLen))
    if v < 0:
        raise _lib.ErrInvalidBlock("ErrInvalidBlock")
    return int(v)


def DecodeSize(totalSize: int, blockLen: int = DefaultBlockSize) -> int:
    """util.go:59-65."""
    v = _lib.lib().cfsec_crc32block_decode_size(int(totalSize), int(blockLen))
    if v < 0:
        raise _lib.ErrInvalidBlock("ErrInvalidBlock")
    return int(v)


def _mem_of(x):
    if _is_torch(x):
        if not x.is_cuda:
            raise TypeError("torch buffers must live on a HIP device")
        return _lib.MEM_DEVICE, x.device.index
    if not (isinstance(x, np.ndarray) and x.dtype == np.uint8 and x.ndim == 1 and x.flags.c_contiguous):
        raise TypeError("host buffers must be 1-D contiguous uint8 numpy arrays")
    return _lib.MEM_HOST, -1


def _empty_like(x, n: int):
    if _is_torch(x):
        import torch
        return torch.empty(n, dtype=torch.uint8, device=x.device)
    return np.empty(n, np.uint8)


def Encode(src, size: int | None = None, block_len: int = DefaultBlockSize, dst=None, stream=None):
    """Frame the first `size` bytes of src (default: all).  Returns (framed, shard_crc)."""
    size = _nbytes(src) if size is None else int(size)
    if size > _nbytes(src):
        raise _lib.ErrShortData("ErrShortData")  # the reader ran dry: encode.go:97-99 ReaderError
    total = EncodeSize(size, block_len)
    mem, dev = _mem_of(src)
    if dst is None:
        dst = _empty_like(src, total)
    elif _nbytes(dst) < total or _mem_of(dst) != (mem, dev):
        raise _lib.ErrInvalidArg("ErrInvalidArg: dst too small or in another memory space / on another device")
    crc = ctypes.c_uint32(0)
    _lib.check(_lib.lib().cfsec_crc32block_encode(_ptr(src) if size else None, size, block_len,
                                                  _ptr(dst) if total else None, ctypes.byref(crc), mem, dev,
                                                  stream_ptr(stream, src)))
    return dst, int(crc.value)


def Decode(src, size: int, from_: int = 0, to: int | None = None, block_len: int = DefaultBlockSize, dst=None,
           stream=None):
    """Payload bytes [from_, to) of a framed object whose payload is `size` bytes; every block
    holding them is checked (ErrMismatchedCrc; the exception's .block is the first bad block)."""
    to = size if to is None else int(to)
    mem, dev = _mem_of(src)
    n = to - from_
    if dst is None:
        dst = _empty_like(src, max(n, 0))
    elif n > 0 and (_nbytes(dst) < n or _mem_of(dst) != (mem, dev)):
        raise _lib.ErrInvalidArg("ErrInvalidArg: dst too small or in another memory space / on another device")
    bad = ctypes.c_int64(-1)
    # the framed length bounds every read: a short object is ErrShortData (the reference's
    # SectionReader: io.ErrUnexpectedEOF), never a read past the buffer
    st = _lib.lib().cfsec_crc32block_decode(_ptr(src) if _nbytes(src) else None, _nbytes(src), int(size),
                                           int(block_len), int(from_), int(to), _ptr(dst) if n > 0 else None,
                                           ctypes.byref(bad), mem, dev, stream_ptr(stream, src))
    if st == _lib.ErrMismatchedCrc.status:
        e = _lib.ErrMismatchedCrc(f"ErrMismatchedCrc: block {bad.value}")
        e.block = int(bad.value)
        raise e
    _lib.check(st)
    return dst


def encode_batch(srcs, dsts, size: int, block_len: int = DefaultBlockSize, shard_crcs_ptr=None, stream=None,
                 device: int = -1):
    """cfsec_crc32block_encode_batch: frame n device payloads of `size` bytes (pointer lists) into
    n framed buffers; shard_crcs_ptr (device, n uint32) receives each payload's ChecksumIEEE.
    Asynchronous on `stream`."""
    _lib.check(_lib.lib().cfsec_crc32block_encode_batch(ptr_array(srcs), ptr_array(dsts), len(srcs), int(size),
                                                        int(block_len), shard_crcs_ptr, _batch_stream(stream, device)))


def _batch_stream(stream, device):
    if stream is None:
        from .reedsolomon import _current_device
        return stream_ptr(None, device=device if device >= 0 else _current_device())
    return stream_ptr(stream)


def decode_batch(srcs, dsts, size: int, bad_ptr: int, from_: int = 0, to: int | None = None,
                 block_len: int = DefaultBlockSize, stream=None, src_len: int | None = None, device: int = -1):
    """cfsec_crc32block_decode_batch: check and unframe payload [from_, to) of n framed device
    objects of at least src_len bytes each (default: EncodeSize(size)); bad_ptr (device, n uint32)
    receives per object the first bad block or 0xFFFFFFFF."""
    to = size if to is None else int(to)
    src_len = EncodeSize(size, block_len) if src_len is None else int(src_len)
    _lib.check(_lib.lib().cfsec_crc32block_decode_batch(ptr_array(srcs), src_len, ptr_array(dsts) if dsts else None,
                                                        len(srcs), int(size), int(block_len), int(from_), to,
                                                        bad_ptr, _batch_stream(stream, device)))
