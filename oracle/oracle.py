"""TEST INFRASTRUCTURE: ctypes front end of the CPU oracle (oracle/gf_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module; the product package (chubaofs_amd) never does.  Every function here is
the checker, restating klauspost/reedsolomon v1.11.7 (see gf_oracle.c header for
the file:line map).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

P_u8 = ctypes.POINTER(ctypes.c_uint8)


def build() -> None:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.oracle_tables.argtypes = [ctypes.c_void_p] * 7
        L.oracle_gal_mul.argtypes = [ctypes.c_uint8, ctypes.c_uint8]
        L.oracle_gal_mul.restype = ctypes.c_uint8
        L.oracle_gal_exp.argtypes = [ctypes.c_uint8, ctypes.c_int]
        L.oracle_gal_exp.restype = ctypes.c_uint8
        L.oracle_invert.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_build_matrix.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        for fn in ("oracle_encode",):
            getattr(L, fn).argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.oracle_verify.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                    ctypes.POINTER(ctypes.c_int)]
        L.oracle_reconstruct.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_void_p]
        L.oracle_crc32_ieee.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        L.oracle_crc32_ieee.restype = ctypes.c_uint32
        L.oracle_crc32_update.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
        L.oracle_crc32_update.restype = ctypes.c_uint32
        _LIB = L
    return _LIB


def tables() -> dict:
    t = {
        "logTable": np.zeros(256, np.uint8),
        "expTable": np.zeros(510, np.uint8),
        "invTable": np.zeros(256, np.uint8),
        "mulTable": np.zeros((256, 256), np.uint8),
        "mulTableLow": np.zeros((256, 16), np.uint8),
        "mulTableHigh": np.zeros((256, 16), np.uint8),
        "gf2p811dMulMatrices": np.zeros(256, np.uint64),
    }
    lib().oracle_tables(*[a.ctypes.data for a in t.values()])
    return t


def gal_mul(a: int, b: int) -> int:
    return lib().oracle_gal_mul(a, b)


def build_matrix(k: int, total: int) -> np.ndarray:
    out = np.zeros((total, k), np.uint8)
    err = lib().oracle_build_matrix(k, total, out.ctypes.data)
    assert err == 0, err
    return out


def invert(mat: np.ndarray):
    mat = np.ascontiguousarray(mat, np.uint8)
    n = mat.shape[0]
    out = np.zeros((n, n), np.uint8)
    err = lib().oracle_invert(n, mat.ctypes.data, out.ctypes.data)
    return err, out


def _ptrs(shards):
    arr = (ctypes.c_void_p * len(shards))()
    for i, s in enumerate(shards):
        arr[i] = s.ctypes.data if s is not None and s.size else 0
    return arr


def _lens(shards, lens=None):
    if lens is None:
        lens = [0 if s is None else s.size for s in shards]
    return (ctypes.c_size_t * len(shards))(*lens)


def encode(k: int, m: int, shards: list) -> int:
    """shards: list of k+m uint8 numpy arrays; parity rows overwritten."""
    return lib().oracle_encode(k, m, _ptrs(shards), _lens(shards), len(shards))


def verify(k: int, m: int, shards: list):
    ok = ctypes.c_int(0)
    err = lib().oracle_verify(k, m, _ptrs(shards), _lens(shards), len(shards), ctypes.byref(ok))
    return err, bool(ok.value)


def reconstruct(k: int, m: int, shards: list, present: list, data_only: bool = False):
    """shards: k+m equal-size buffers; present[i] False marks missing (buffer is scratch).

    Returns (err, filled) where filled[i] is True for shards written."""
    lens = [s.size if p else 0 for s, p in zip(shards, present)]
    lens_c = _lens(shards, lens)
    arr = (ctypes.c_void_p * len(shards))(*[s.ctypes.data for s in shards])
    dec = np.zeros((k, k), np.uint8)
    err = lib().oracle_reconstruct(k, m, arr, lens_c, len(shards), int(data_only), dec.ctypes.data)
    filled = [(not p) and lens_c[i] != 0 for i, p in enumerate(present)]
    return err, filled


def crc32_ieee(buf) -> int:
    b = np.ascontiguousarray(np.frombuffer(bytes(buf), np.uint8) if not isinstance(buf, np.ndarray) else buf)
    return lib().oracle_crc32_ieee(b.ctypes.data, b.size)


def encode_matrix_rows(k: int, total: int) -> np.ndarray:
    return build_matrix(k, total)[k:]


# ---- klauspost-strategy SIMD baseline (bench.py cpu_baseline leg) ----
def _simd():
    L = lib()
    if not getattr(L, "_simd_ready", False):
        L.cpu_code_some_shards.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int]
        L.cpu_code_some_shards.restype = ctypes.c_int
        L.cpu_has_gfni.restype = ctypes.c_int
        L.cpu_has_avx2.restype = ctypes.c_int
        L._simd_ready = True
    return L


def simd_features() -> dict:
    L = _simd()
    return {"gfni": bool(L.cpu_has_gfni()), "avx2": bool(L.cpu_has_avx2())}


def simd_code(rows: np.ndarray, inputs: list, outputs: list, threads: int, force: int = 0) -> int:
    """outputs = rows x inputs with the AVX2/GFNI tile kernels; returns 1 (AVX2) or 2 (GFNI)."""
    rows = np.ascontiguousarray(rows, np.uint8)
    m, k = rows.shape
    ins = (ctypes.c_void_p * k)(*[a.ctypes.data for a in inputs])
    outs = (ctypes.c_void_p * m)(*[a.ctypes.data for a in outputs])
    ret = _simd().cpu_code_some_shards(rows.ctypes.data, k, m, ins, outs, inputs[0].size, threads, force)
    if ret < 0:
        raise RuntimeError("SIMD path unavailable on this CPU")
    return ret


# ---- crc32block framing (blobstore/common/crc32block), restated over the CRC above ----
CRC32BLOCK_DEFAULT = 64 * 1024  # defaultCrc32BlockSize, block.go:22-24


def crc32block_valid_len(block_len: int) -> bool:
    """isValidBlockLen, util.go:34-36 (baseBlockLen = 1 << 12)."""
    return block_len > 0 and block_len % 4096 == 0


def crc32block_encode_size(size: int, block_len: int) -> int:
    """EncodeSize, util.go:50-57."""
    if not crc32block_valid_len(block_len):
        raise ValueError("ErrInvalidBlock")
    payload = block_len - 4
    return size + 4 * ((size + payload - 1) // payload)


def crc32block_decode_size(total: int, block_len: int) -> int:
    """DecodeSize, util.go:59-65."""
    if not crc32block_valid_len(block_len):
        raise ValueError("ErrInvalidBlock")
    return total - 4 * ((total + block_len - 1) // block_len)


def crc32block_encode(payload: np.ndarray, block_len: int = CRC32BLOCK_DEFAULT) -> np.ndarray:
    """limitEncoderReader.nextBlock (encode.go:87-109) + blockUnit.writeCrc (block.go:46-49): each
    block is [LE crc32.ChecksumIEEE(payload piece)][payload piece of <= block_len - 4 bytes]."""
    payload = np.ascontiguousarray(payload, np.uint8)
    out = np.empty(crc32block_encode_size(payload.size, block_len), np.uint8)
    P = block_len - 4
    for b, q in enumerate(range(0, payload.size, P)):
        piece = payload[q:q + P]
        o = b * block_len
        out[o:o + 4] = np.frombuffer(int(crc32_ieee(piece)).to_bytes(4, "little"), np.uint8)
        out[o + 4:o + 4 + piece.size] = piece
    return out


def crc32block_decode(framed: np.ndarray, size: int, from_: int, to: int, block_len: int = CRC32BLOCK_DEFAULT):
    """Decoder.Reader(from, to) read to EOF (decode.go:122-146): blockReader.nextBlock checks each
    block it reads (decode.go:85-108) starting at the block holding `from`; rangeReader skips
    from % payload bytes (reading -- and checking -- that block even when from == to) and stops
    after to - from bytes.  Returns (bytes, index of the first bad block or -1)."""
    P = block_len - 4
    if not crc32block_valid_len(block_len) or not 0 <= from_ <= to <= size:
        raise ValueError("invalid range")
    b0 = from_ // P
    b1 = (to - 1) // P if from_ < to else (b0 if from_ % P else b0 - 1)
    got = bytearray()
    for b in range(b0, b1 + 1):
        plen = min(P, size - b * P)
        blk = framed[b * block_len:b * block_len + 4 + plen]
        if int.from_bytes(bytes(blk[:4]), "little") != crc32_ieee(np.ascontiguousarray(blk[4:])):
            return np.frombuffer(bytes(got), np.uint8), b
        lo, hi = max(from_, b * P), min(to, b * P + plen)
        if lo < hi:
            got += bytes(blk[4 + lo - b * P:4 + hi - b * P])
    return np.frombuffer(bytes(got), np.uint8), -1
