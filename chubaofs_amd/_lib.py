"""ctypes binding of libcfsec.so (include/cfsec.h).

The library is the product: every Encode/Verify/Reconstruct below runs the gfx950
kernels in chubaofs_amd/csrc.  There is no CPU fallback -- if the shared object is
missing, importing this module raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# CFSEC_LIB_PATH: another build of the same library (A/B probes of kernel variants)
LIB_PATH = os.environ.get("CFSEC_LIB_PATH") or os.path.join(_HERE, "libcfsec.so")

MEM_HOST = 0
MEM_DEVICE = 1


class Shard(ctypes.Structure):
    """One Go []byte: {data, len, cap}."""

    _fields_ = [("data", ctypes.c_void_p), ("len", ctypes.c_size_t), ("cap", ctypes.c_size_t)]


class TacticC(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("n", "m", "l", "az_count", "put_quorum", "get_quorum", "min_shard_size")]


# ---- errors: 1:1 with the Go sentinels (see include/cfsec.h) ----
class CfsecError(Exception):
    status = -1


def _mk(name, code, doc):
    return type(name, (CfsecError,), {"status": code, "__doc__": doc})


ErrTooFewShards = _mk("ErrTooFewShards", 1, "reedsolomon.ErrTooFewShards")
ErrShardNoData = _mk("ErrShardNoData", 2, "reedsolomon.ErrShardNoData")
ErrShardSize = _mk("ErrShardSize", 3, "reedsolomon.ErrShardSize")
ErrInvShardNum = _mk("ErrInvShardNum", 4, "reedsolomon.ErrInvShardNum")
ErrMaxShardNum = _mk("ErrMaxShardNum", 5, "reedsolomon.ErrMaxShardNum")
ErrShortData = _mk("ErrShortData", 6, "reedsolomon.ErrShortData / ec.ErrShortData")
ErrReconstructRequired = _mk("ErrReconstructRequired", 7, "reedsolomon.ErrReconstructRequired")
ErrSingular = _mk("ErrSingular", 8, "reedsolomon errSingular")
ErrInvalidCodeMode = _mk("ErrInvalidCodeMode", 9, "ec.ErrInvalidCodeMode")
ErrVerify = _mk("ErrVerify", 10, "ec.ErrVerify")
ErrInvalidShards = _mk("ErrInvalidShards", 11, "ec.ErrInvalidShards")
ErrInvalidArg = _mk("ErrInvalidArg", 12, "boundary misuse")
ErrDevice = _mk("ErrDevice", 13, "HIP runtime failure")
ErrNotSupported = _mk("ErrNotSupported", 14, "reedsolomon.ErrNotSupported")
ErrInvalidBlock = _mk("ErrInvalidBlock", 15, "crc32block.ErrInvalidBlock")
ErrMismatchedCrc = _mk("ErrMismatchedCrc", 16, "crc32block.ErrMismatchedCrc")

_BY_CODE = {c.status: c for c in (
    ErrTooFewShards, ErrShardNoData, ErrShardSize, ErrInvShardNum, ErrMaxShardNum, ErrShortData,
    ErrReconstructRequired, ErrSingular, ErrInvalidCodeMode, ErrVerify, ErrInvalidShards,
    ErrInvalidArg, ErrDevice, ErrNotSupported, ErrInvalidBlock, ErrMismatchedCrc)}


def check(status: int) -> None:
    if status == 0:
        return
    cls = _BY_CODE.get(status, CfsecError)
    msg = cls.__name__
    if status in (ErrDevice.status, ErrInvalidArg.status):
        detail = lib().cfsec_last_error().decode()
        if detail:
            msg += ": " + detail
    raise cls(msg)


# ---- symbol table: every entry point of include/cfsec.h ----
_V, _I, _S, _P = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.POINTER
P_SHARD = ctypes.POINTER(Shard)
SIGNATURES = {
    "cfsec_version": ([], ctypes.c_char_p),
    "cfsec_last_error": ([], ctypes.c_char_p),
    "cfsec_status_name": ([_I], ctypes.c_char_p),
    "cfsec_device_count": ([], _I),
    "cfsec_set_sync_poll": ([_I], _I),
    "cfsec_rs_new": ([_I, _I, _I, _P(_V)], _I),
    "cfsec_rs_free": ([_V], None),
    "cfsec_rs_data_shards": ([_V], _I),
    "cfsec_rs_parity_shards": ([_V], _I),
    "cfsec_rs_matrix": ([_V, _V, _S], _I),
    "cfsec_rs_encode": ([_V, P_SHARD, _I, _I, _V], _I),
    "cfsec_rs_verify": ([_V, P_SHARD, _I, _I, _V, _P(_I)], _I),
    "cfsec_rs_reconstruct": ([_V, P_SHARD, _I, _I, _V], _I),
    "cfsec_rs_reconstruct_data": ([_V, P_SHARD, _I, _I, _V], _I),
    "cfsec_rs_split": ([_V, _V, _S, _S, P_SHARD, _V, _S, _P(_S)], _I),
    "cfsec_rs_join": ([_V, _V, _S, P_SHARD, _I, _S], _I),
    "cfsec_rs_encode_batch": ([_V, _V, _S, _I, _V], _I),
    "cfsec_rs_verify_batch": ([_V, _V, _S, _I, _V, _V], _I),
    "cfsec_rs_reconstruct_batch": ([_V, _V, _S, _I, _V, _I, _I, _V], _I),
    "cfsec_rs_encode_crc": ([_V, P_SHARD, _I, _I, _V, _V], _I),
    "cfsec_rs_encode_crc_batch": ([_V, _V, _S, _I, _V, _V], _I),
    "cfsec_rs_reconstruct_crc_batch": ([_V, _V, _S, _I, _V, _I, _I, _V, _V], _I),
    "cfsec_rs_set_devices": ([_V, _V, _I], _I),
    "cfsec_batch_partition": ([_V, _I, _I, _V], _I),
    "cfsec_rs_encode_stripes": ([_V, P_SHARD, _I, _I, _V], _I),
    "cfsec_rs_verify_stripes": ([_V, P_SHARD, _I, _I, _V], _I),
    "cfsec_rs_reconstruct_stripes": ([_V, P_SHARD, _I, _I, _I, _V], _I),
    "cfsec_codemode_tactic": ([_I, _P(TacticC)], _I),
    "cfsec_ec_new": ([_P(TacticC), _I, _I, _I, _P(_V)], _I),
    "cfsec_ec_free": ([_V], None),
    "cfsec_ec_encode": ([_V, P_SHARD, _I, _I, _V], _I),
    "cfsec_ec_reconstruct": ([_V, P_SHARD, _I, _V, _I, _I, _V], _I),
    "cfsec_ec_reconstruct_data": ([_V, P_SHARD, _I, _V, _I, _I, _V], _I),
    "cfsec_ec_verify": ([_V, P_SHARD, _I, _I, _V, _P(_I)], _I),
    "cfsec_ec_shards_in_idc": ([_V, _I, _V, _I, _P(_I)], _I),
    "cfsec_ec_repair_rows": ([_V, _V, _I, _V, _I, _V, _V], _I),
    "cfsec_ec_matvec_batch": ([_V, _V, _I, _V, _S, _I, _V], _I),
    "cfsec_ec_set_devices": ([_V, _V, _I], _I),
    "cfsec_ec_encode_batch": ([_V, P_SHARD, _I, _I, _I, _V], _I),
    "cfsec_ec_reconstruct_batch": ([_V, P_SHARD, _I, _I, _V, _V, _I, _I, _V], _I),
    "cfsec_ec_reconstruct_batch_async": ([_V, P_SHARD, _I, _I, _V, _V, _I, _V, _V, _V, _V], _I),
    "cfsec_ec_encode_batch_async": ([_V, P_SHARD, _I, _I, _V, _V, _V, _V], _I),
    "cfsec_ec_encode_batch_crc": ([_V, P_SHARD, _I, _I, _I, _V, _V], _I),
    "cfsec_ec_reconstruct_batch_crc": ([_V, P_SHARD, _I, _I, _V, _V, _I, _I, _V, _V], _I),
    "cfsec_rs_encode_contig": ([_V, _V, _S, _S, _I, _I, _V], _I),
    "cfsec_rs_verify_contig": ([_V, _V, _S, _S, _I, _I, _V, _P(_I)], _I),
    "cfsec_rs_reconstruct_contig": ([_V, _V, _S, _S, _I, _V, _I, _I, _I, _V], _I),
    "cfsec_ec_encode_contig": ([_V, _V, _S, _S, _I, _I, _V], _I),
    "cfsec_ec_verify_contig": ([_V, _V, _S, _S, _I, _I, _V, _P(_I)], _I),
    "cfsec_ec_reconstruct_contig": ([_V, _V, _S, _S, _I, _V, _I, _I, _I, _V], _I),
    "cfsec_ec_encode_batch_contig": ([_V, _V, _S, _S, _S, _I, _I, _I, _V, _V], _I),
    "cfsec_ec_reconstruct_batch_contig": ([_V, _V, _V, _V, _I, _I, _V, _V, _I, _I, _V, _V], _I),
    "cfsec_crc32_ieee_batch": ([_V, _S, _I, _V, _I, _V], _I),
    "cfsec_crc32_combine": ([ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int64], ctypes.c_uint32),
    "cfsec_crc32_shift": ([_V, _I, ctypes.c_int64], _I),
    "cfsec_stream_copy": ([_V, _V, _S, _V], _I),
    "cfsec_host_alloc": ([_S, _P(_V)], _I),
    "cfsec_host_free": ([_V], _I),
    "cfsec_crc32block_encode_size": ([ctypes.c_int64, ctypes.c_int64], ctypes.c_int64),
    "cfsec_crc32block_decode_size": ([ctypes.c_int64, ctypes.c_int64], ctypes.c_int64),
    "cfsec_crc32block_encode": ([_V, ctypes.c_int64, ctypes.c_int64, _V, _P(ctypes.c_uint32), _I, _I, _V], _I),
    "cfsec_crc32block_decode": ([_V, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                 ctypes.c_int64, _V, _P(ctypes.c_int64), _I, _I, _V], _I),
    "cfsec_crc32block_encode_batch": ([_V, _V, _I, ctypes.c_int64, ctypes.c_int64, _V, _V], _I),
    "cfsec_crc32block_decode_batch": ([_V, ctypes.c_int64, _V, _I, ctypes.c_int64, ctypes.c_int64,
                                       ctypes.c_int64, ctypes.c_int64, _V, _V], _I),
}

_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: the HIP engine is not built "
                "(run `python -c 'import __graft_entry__ as g; g.build()'`); there is no CPU fallback")
        # One HIP runtime per process: PyTorch ships its own libamdhip64.so.7 / libhsa-runtime64.so.1
        # under the same SONAMEs as /opt/rocm's, and whichever loads first serves both.  Load
        # torch's first when torch is installed -- with /opt/rocm's loaded first, torch finds no
        # device (seen on MI355X); the engine runs on either runtime.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        for name, (args, res) in SIGNATURES.items():
            if os.environ.get("CFSEC_LIB_PATH") and not hasattr(L, name):
                continue  # an older probe build (A/B of an earlier round's library): newer entry points absent
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _LIB = L
    return _LIB


def device_count() -> int:
    return lib().cfsec_device_count()


class _Pinned:
    """Owner of one cfsec_host_alloc block; frees it when the last numpy view is gone."""

    def __init__(self, size: int):
        p = ctypes.c_void_p()
        check(lib().cfsec_host_alloc(size, ctypes.byref(p)))
        self.ptr, self.size = p.value, size

    def __del__(self):
        if getattr(self, "ptr", None):
            lib().cfsec_host_free(self.ptr)
            self.ptr = None


def pinned_empty(size: int):
    """A uint8 numpy array in page-locked host memory (cfsec_host_alloc): host-memory calls on it
    DMA straight to HBM.  The array keeps the allocation alive."""
    import numpy as np

    if size == 0:
        return np.zeros(0, np.uint8)
    owner = _Pinned(size)
    buf = (ctypes.c_uint8 * size).from_address(owner.ptr)
    arr = np.frombuffer(buf, dtype=np.uint8)
    buf._cfsec_owner = owner  # the ctypes buffer (referenced by arr.base) holds the owner
    return arr


def batch_partition(nbytes, ndev: int):
    """cfsec_batch_partition: the device index each stripe of a host batch runs on."""
    import numpy as np

    b = np.ascontiguousarray(np.asarray(nbytes, np.uint64))
    out = np.zeros(max(len(b), 1), np.int32)
    check(lib().cfsec_batch_partition(b.ctypes.data if len(b) else None, len(b), ndev, out.ctypes.data))
    return [int(x) for x in out[:len(b)]]
