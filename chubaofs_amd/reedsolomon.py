"""reedsolomon -- the engine seam: mirror of reedsolomon.Encoder
(vendor/github.com/klauspost/reedsolomon/reedsolomon.go:25-131) backed by
libcfsec.so's cfsec_rs_* entry points (gfx950 kernels).

    enc = New(12, 4)
    enc.Encode(shards)            # shards: 16 equal-length uint8 buffers
    ok = enc.Verify(shards)
    shards[0] = shards[0][:0]     # mark missing
    enc.Reconstruct(shards)
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._shards import BatchMarshal, Marshal, ptr_array, shard_size, stream_ptr


class ReedSolomon:
    def __init__(self, data_shards: int, parity_shards: int, device: int = -1):
        L = _lib.lib()
        h = ctypes.c_void_p()
        _lib.check(L.cfsec_rs_new(data_shards, parity_shards, device, ctypes.byref(h)))
        self._h = h
        self._L = L
        self.data_shards = data_shards
        self.parity_shards = parity_shards
        self.total_shards = data_shards + parity_shards
        self.device = device if device >= 0 else _current_device()

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._L.cfsec_rs_free(h)
            self._h = None

    # -- KRS Encoder methods used by CubeFS --
    def Encode(self, shards, stream=None) -> None:
        m = Marshal(shards)
        _lib.check(self._L.cfsec_rs_encode(self._h, m.ptr(), m.n, m.mem, stream_ptr(stream, m.like)))

    def EncodeCRC(self, shards, stream=None):
        """Encode + crc32.ChecksumIEEE of every shard, fused (cfsec_rs_encode_crc); returns the
        n checksums (what access computes per shard after Encode, stream_put.go:249-253)."""
        m = Marshal(shards)
        out = (ctypes.c_uint32 * max(m.n, 1))()
        _lib.check(self._L.cfsec_rs_encode_crc(self._h, m.ptr(), m.n, m.mem, stream_ptr(stream, m.like), out))
        return [int(out[i]) for i in range(m.n)]

    def Verify(self, shards, stream=None) -> bool:
        m = Marshal(shards)
        ok = ctypes.c_int(0)
        _lib.check(self._L.cfsec_rs_verify(self._h, m.ptr(), m.n, m.mem, stream_ptr(stream, m.like), ctypes.byref(ok)))
        return bool(ok.value)

    def _reconstruct(self, fn, shards, stream):
        m = Marshal(shards, fill_size=shard_size(shards))
        st = fn(self._h, m.ptr(), m.n, m.mem, stream_ptr(stream, m.like))
        m.writeback()
        _lib.check(st)

    def Reconstruct(self, shards, stream=None) -> None:
        self._reconstruct(self._L.cfsec_rs_reconstruct, shards, stream)

    def ReconstructData(self, shards, stream=None) -> None:
        self._reconstruct(self._L.cfsec_rs_reconstruct_data, shards, stream)

    def Split(self, data: np.ndarray, length: int | None = None):
        """Split data[:length] (cap = data.size) into views, KRS/reedsolomon.go:1574-1632."""
        if length is None:
            length = int(data.size)
        out = (_lib.Shard * self.total_shards)()
        need = ctypes.c_size_t(0)
        ptr = data.ctypes.data if data.size else None
        st = self._L.cfsec_rs_split(self._h, ptr, length, int(data.size), out, None, 0, ctypes.byref(need))
        pad = None
        if st == _lib.ErrInvalidArg.status and need.value:
            pad = np.zeros(need.value, np.uint8)
            st = self._L.cfsec_rs_split(self._h, ptr, length, int(data.size), out, pad.ctypes.data,
                                        pad.size, ctypes.byref(need))
        _lib.check(st)
        views = []
        for i in range(self.total_shards):
            for src in (data, pad):
                if src is None or not src.size:
                    continue
                off = out[i].data - src.ctypes.data
                if 0 <= off < src.size:
                    views.append(src[off:off + out[i].len])
                    break
            else:
                raise RuntimeError("split returned a pointer outside its buffers")
        return views

    def Join(self, dst, shards, out_size: int) -> None:
        """Write out_size bytes of the data shards to dst (a writer or bytearray)."""
        m = Marshal(list(shards))
        for i, s in enumerate(shards):  # only a Go nil slice (None) is "missing" for Join
            if s is None:
                m.arr[i].data = None
            elif m.arr[i].data is None:
                m.arr[i].data = 1  # non-nil empty slice; never dereferenced
        buf = np.zeros(max(out_size, 1), np.uint8)
        _lib.check(self._L.cfsec_rs_join(self._h, buf.ctypes.data, buf.size, m.ptr(), m.n, out_size))
        data = buf[:out_size].tobytes()
        if hasattr(dst, "write"):
            dst.write(data)
        else:
            dst.extend(data)

    # -- stripe batches over the handle's devices (cfsec_rs_*_stripes) --
    def SetDevices(self, devices) -> None:
        """Spread stripe batches over these HIP devices (default: the handle's own)."""
        arr = (ctypes.c_int * len(devices))(*devices)
        _lib.check(self._L.cfsec_rs_set_devices(self._h, arr, len(devices)))

    def _stripes(self, fn, stripes, fill, *extra):
        bm = BatchMarshal(stripes, self.total_shards, fill=fill)
        status = (ctypes.c_int * max(len(stripes), 1))()
        st = fn(self._h, bm.arr, len(stripes), *extra, bm.mem, status)
        bm.writeback()
        _lib.check(st)
        return [int(status[i]) for i in range(len(stripes))]

    def EncodeStripes(self, stripes):
        """Encode every stripe (each a list of total_shards buffers, sizes may differ per stripe);
        returns one status code per stripe (0 = ok, else the code Encode would raise)."""
        return self._stripes(self._L.cfsec_rs_encode_stripes, stripes, False)

    def VerifyStripes(self, stripes):
        """Per stripe: 0 when Verify holds, ErrVerify.status when it returns false, else the error."""
        return self._stripes(self._L.cfsec_rs_verify_stripes, stripes, False)

    def ReconstructStripes(self, stripes, verify: bool = True):
        """Reconstruct (+ Verify) every stripe in one fused pass per stripe; missing entries (None or
        empty) are replaced in the lists by the rebuilt shards.  Per-stripe status codes."""
        return self._stripes(self._L.cfsec_rs_reconstruct_stripes, stripes, True, int(verify))

    # -- helpers / GPU batch API --
    def matrix(self) -> np.ndarray:
        out = np.zeros((self.total_shards, self.data_shards), np.uint8)
        _lib.check(self._L.cfsec_rs_matrix(self._h, out.ctypes.data, out.size))
        return out

    def encode_batch(self, ptrs, shard_len: int, nstripes: int, stream=None) -> None:
        _lib.check(self._L.cfsec_rs_encode_batch(self._h, ptr_array(ptrs), shard_len, nstripes,
                                                 stream_ptr(stream, device=self.device)))

    def verify_batch(self, ptrs, shard_len: int, nstripes: int, flags_ptr: int, stream=None) -> None:
        _lib.check(self._L.cfsec_rs_verify_batch(self._h, ptr_array(ptrs), shard_len, nstripes,
                                                 flags_ptr, stream_ptr(stream, device=self.device)))

    def reconstruct_batch(self, ptrs, shard_len: int, nstripes: int, erased, data_only=False,
                          stream=None) -> None:
        er = (ctypes.c_int * max(len(erased), 1))(*erased)
        _lib.check(self._L.cfsec_rs_reconstruct_batch(self._h, ptr_array(ptrs), shard_len, nstripes, er,
                                                      len(erased), int(data_only), stream_ptr(stream, device=self.device)))

    def encode_crc_batch(self, ptrs, shard_len: int, nstripes: int, crcs_ptr: int, stream=None) -> None:
        """encode_batch + crc32.ChecksumIEEE of every shard into the device uint32 array at
        crcs_ptr, [stripe][shard] (access/stream_put.go:249-253), fused where supported."""
        _lib.check(self._L.cfsec_rs_encode_crc_batch(self._h, ptr_array(ptrs), shard_len, nstripes, crcs_ptr,
                                                     stream_ptr(stream, device=self.device)))

    def reconstruct_crc_batch(self, ptrs, shard_len: int, nstripes: int, erased, crcs_ptr: int,
                              data_only=False, stream=None) -> None:
        """reconstruct_batch + crc32.ChecksumIEEE of each rebuilt shard ([stripe][shard]; other
        words 0)."""
        er = (ctypes.c_int * max(len(erased), 1))(*erased)
        _lib.check(self._L.cfsec_rs_reconstruct_crc_batch(self._h, ptr_array(ptrs), shard_len, nstripes, er,
                                                          len(erased), int(data_only), crcs_ptr,
                                                          stream_ptr(stream, device=self.device)))


def _current_device() -> int:
    """The HIP device a handle created with device=-1 binds to (the calling thread's current one)."""
    import sys
    torch = sys.modules.get("torch")
    if torch is not None and torch.cuda.is_initialized():
        return torch.cuda.current_device()
    return 0


def New(data_shards: int, parity_shards: int, device: int = -1) -> ReedSolomon:
    """reedsolomon.New with default options (KRS/reedsolomon.go:413)."""
    return ReedSolomon(data_shards, parity_shards, device)


def crc32_ieee_batch(ptrs, shard_len: int, device: int = -1, stream=None):
    """crc32.ChecksumIEEE of each device shard (list of device pointers)."""
    L = _lib.lib()
    out = (ctypes.c_uint32 * max(len(ptrs), 1))()
    dev = device if device >= 0 else _current_device()
    _lib.check(L.cfsec_crc32_ieee_batch(ptr_array(ptrs), shard_len, len(ptrs), out, device,
                                        stream_ptr(stream, device=dev)))
    return [int(out[i]) for i in range(len(ptrs))]
