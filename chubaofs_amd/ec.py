"""ec -- mirror of blobstore/common/ec (encoder.go, lrcencoder.go, buf.go) over
libcfsec.so's cfsec_ec_* entry points.  Method names, argument meaning and
errors follow the Go interface so the tests read like encoder_test.go:

    enc = NewEncoder(Config(CodeMode=codemode.GetTactic(codemode.EC6P10L2), EnableVerify=True))
    shards = enc.Split(data)
    enc.Encode(shards)
    enc.Reconstruct(shards, [0, 17])
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import ErrShortData, ErrInvalidCodeMode, ErrVerify, ErrInvalidShards  # noqa: F401 (re-export)
from ._shards import BatchMarshal, Marshal, shard_size, stream_ptr
from .codemode import Tactic
from .reedsolomon import ReedSolomon

DEFAULT_CONCURRENCY = 100  # encoder.go:29


@dataclass
class Config:
    """ec.Config (encoder.go:65-69)."""

    CodeMode: Tactic
    EnableVerify: bool = False
    Concurrency: int = 0


def _tactic_c(t: Tactic) -> _lib.TacticC:
    return _lib.TacticC(t.N, t.M, t.L, t.AZCount, t.PutQuorum, t.GetQuorum, t.MinShardSize)


class Encoder:
    """ec.Encoder (encoder.go:41-62); LRC modes behave as lrcEncoder (lrcencoder.go)."""

    def __init__(self, cfg: Config, device: int = -1):
        L = _lib.lib()
        h = ctypes.c_void_p()
        tc = _tactic_c(cfg.CodeMode)
        _lib.check(L.cfsec_ec_new(ctypes.byref(tc), int(cfg.EnableVerify), cfg.Concurrency, device,
                                  ctypes.byref(h)))
        self._h, self._L, self.cfg = h, L, cfg
        t = cfg.CodeMode
        self._engine = ReedSolomon(t.N, t.M, device)  # host-side Split/Join only

    def __del__(self):
        h = getattr(self, "_h", None)
        if h:
            self._L.cfsec_ec_free(h)
            self._h = None

    @property
    def CodeMode(self) -> Tactic:
        return self.cfg.CodeMode

    # -- coding --
    def Encode(self, shards, stream=None) -> None:
        m = Marshal(shards, fill_size=shard_size(shards))
        st = self._L.cfsec_ec_encode(self._h, m.ptr(), m.n, m.mem, stream_ptr(stream, m.like))
        m.writeback()
        _lib.check(st)

    def _recon(self, fn, shards, badIdx, stream):
        m = Marshal(shards, fill_size=shard_size(shards))
        bad = (ctypes.c_int * max(len(badIdx), 1))(*badIdx)
        st = fn(self._h, m.ptr(), m.n, bad, len(badIdx), m.mem, stream_ptr(stream, m.like))
        m.writeback()
        _lib.check(st)

    def Reconstruct(self, shards, badIdx, stream=None) -> None:
        self._recon(self._L.cfsec_ec_reconstruct, shards, list(badIdx), stream)

    def ReconstructData(self, shards, badIdx, stream=None) -> None:
        self._recon(self._L.cfsec_ec_reconstruct_data, shards, list(badIdx), stream)

    def Verify(self, shards, stream=None) -> bool:
        m = Marshal(shards)
        ok = ctypes.c_int(0)
        _lib.check(self._L.cfsec_ec_verify(self._h, m.ptr(), m.n, m.mem, stream_ptr(stream, m.like), ctypes.byref(ok)))
        return bool(ok.value)

    # -- batches (blobnode repair loop, work_shard_recover.go:708-771) --
    def SetDevices(self, devices) -> None:
        arr = (ctypes.c_int * len(devices))(*devices)
        _lib.check(self._L.cfsec_ec_set_devices(self._h, arr, len(devices)))

    def EncodeBatch(self, stripes, crcs: bool = False):
        """Encode every stripe (each a list of N+M+L shards; sizes may differ per stripe) in one
        call, EnableVerify included; returns per-stripe status codes, and with crcs=True also
        crc32.ChecksumIEEE of every shard per stripe (cfsec_ec_encode_batch_crc)."""
        n = len(stripes[0]) if stripes else 0
        bm = BatchMarshal(stripes, n, fill=True)
        status = (ctypes.c_int * max(len(stripes), 1))()
        if crcs:
            words = (ctypes.c_uint32 * max(len(stripes) * n, 1))()
            st = self._L.cfsec_ec_encode_batch_crc(self._h, bm.arr, n, len(stripes), bm.mem, status, words)
        else:
            st = self._L.cfsec_ec_encode_batch(self._h, bm.arr, n, len(stripes), bm.mem, status)
        bm.writeback()
        _lib.check(st)
        out = [int(status[i]) for i in range(len(stripes))]
        if crcs:
            return out, [[int(words[s * n + i]) for i in range(n)] for s in range(len(stripes))]
        return out

    def ReconstructBatch(self, bids, badIdx, verify: bool = True, crcs: bool = False):
        """bids: list of shard lists (one per bid, all of one length n); badIdx: one index list per
        bid.  Per bid Reconstruct(shards, bad) then Verify(shards), one batched call; returns the
        per-bid status codes (0 ok, ErrVerify.status when Verify is false, else the error), and with
        crcs=True also per bid the checksums of the shards it rebuilt (0 elsewhere)."""
        if len(bids) != len(badIdx):
            raise ValueError("one bad-index list per bid")
        n = len(bids[0]) if bids else 0
        bm = BatchMarshal(bids, n, fill=True)
        flat = [i for b in badIdx for i in b]
        off = [0]
        for b in badIdx:
            off.append(off[-1] + len(b))
        bad = (ctypes.c_int * max(len(flat), 1))(*flat)
        offs = (ctypes.c_int * len(off))(*off)
        status = (ctypes.c_int * max(len(bids), 1))()
        if crcs:
            words = (ctypes.c_uint32 * max(len(bids) * n, 1))()
            st = self._L.cfsec_ec_reconstruct_batch_crc(self._h, bm.arr, n, len(bids), bad, offs, int(verify),
                                                        bm.mem, status, words)
        else:
            st = self._L.cfsec_ec_reconstruct_batch(self._h, bm.arr, n, len(bids), bad, offs, int(verify), bm.mem,
                                                    status)
        bm.writeback()
        _lib.check(st)
        out = [int(status[i]) for i in range(len(bids))]
        if crcs:
            return out, [[int(words[b * n + i]) for i in range(n)] for b in range(len(bids))]
        return out

    def ReconstructBatchAsync(self, bids, badIdx, flags=None, verify: bool = True, stream=None, crcs=None):
        """cfsec_ec_reconstruct_batch_async: bids of device tensors; enqueues on `stream` (default:
        torch's current stream) and returns the per-bid planning status right away.  flags: a zeroed
        device int32 tensor of len(bids) words; flags[b] != 0 once the stream has passed the call
        where Verify is false.  crcs: optional device int32 tensor of len(bids) * n words for the
        rebuilt shards' checksums."""
        if len(bids) != len(badIdx):
            raise ValueError("one bad-index list per bid")
        n = len(bids[0]) if bids else 0
        bm = BatchMarshal(bids, n, fill=True)
        if bids and bm.mem != _lib.MEM_DEVICE:
            raise TypeError("the asynchronous batch takes device tensors")
        flat = [i for b in badIdx for i in b]
        off = [0]
        for b in badIdx:
            off.append(off[-1] + len(b))
        bad = (ctypes.c_int * max(len(flat), 1))(*flat)
        offs = (ctypes.c_int * len(off))(*off)
        status = (ctypes.c_int * max(len(bids), 1))()
        like = next((x for st in bids for x in st if x is not None and x.numel()), None)
        st = self._L.cfsec_ec_reconstruct_batch_async(self._h, bm.arr, n, len(bids), bad, offs, int(verify), status,
                                                      None if flags is None else flags.data_ptr(),
                                                      None if crcs is None else crcs.data_ptr(),
                                                      stream_ptr(stream, like))
        bm.writeback()
        _lib.check(st)
        return [int(status[i]) for i in range(len(bids))]

    def EncodeBatchAsync(self, stripes, flags=None, stream=None, crcs=None):
        """cfsec_ec_encode_batch_async: as EncodeBatch on device tensors, enqueued on `stream`; with
        EnableVerify a false Verify sets flags[s] (zeroed device int32 tensor) on the stream; crcs:
        optional device int32 tensor of len(stripes) * n words for every shard's checksum."""
        n = len(stripes[0]) if stripes else 0
        bm = BatchMarshal(stripes, n, fill=True)
        if stripes and bm.mem != _lib.MEM_DEVICE:
            raise TypeError("the asynchronous batch takes device tensors")
        status = (ctypes.c_int * max(len(stripes), 1))()
        like = next((x for st in stripes for x in st if x is not None and x.numel()), None)
        st = self._L.cfsec_ec_encode_batch_async(self._h, bm.arr, n, len(stripes), status,
                                                 None if flags is None else flags.data_ptr(),
                                                 None if crcs is None else crcs.data_ptr(), stream_ptr(stream, like))
        bm.writeback()
        _lib.check(st)
        return [int(status[i]) for i in range(len(stripes))]

    # -- slice bookkeeping (host) --
    def Split(self, data, length: int | None = None):
        """encoder.go:153-155 / lrcencoder.go:203-222.  data: uint8 array; data[:length] is the
        payload, data.size its capacity."""
        data = np.asarray(data, np.uint8) if not isinstance(data, np.ndarray) else data
        shards = self._engine.Split(data, length)
        t = self.CodeMode
        if t.L:
            shard_n, shard_len = len(shards), len(shards[0])
            if data.size >= (t.L + shard_n) * shard_len:
                shards += [data[(shard_n + i) * shard_len:(shard_n + i + 1) * shard_len] for i in range(t.L)]
            else:
                shards += [np.zeros(shard_len, np.uint8) for _ in range(t.L)]
        return shards

    def Join(self, dst, shards, outSize: int) -> None:
        t = self.CodeMode
        self._engine.Join(dst, shards[:t.N + t.M] if t.L else shards, outSize)

    def GetDataShards(self, shards):
        return shards[:self.CodeMode.N]

    def GetParityShards(self, shards):
        t = self.CodeMode
        return shards[t.N:t.N + t.M] if t.L else shards[t.N:]

    def GetLocalShards(self, shards):
        t = self.CodeMode
        return shards[t.N + t.M:] if t.L else []

    def GetShardsInIdc(self, shards, idx: int):
        t = self.CodeMode
        if t.L:
            # lrcencoder.go:236-243: a fresh list of the AZ's local stripe
            return [shards[g] for g in self.shards_in_idc(idx)]
        # encoder.go:169-176: Go's append(shards[a:b], shards[c:d]...) writes the parity
        # headers into shards[b:] of the caller's slice (same backing array); kept as is.
        ln, lm = t.N // t.AZCount, t.M // t.AZCount
        b = (idx + 1) * ln
        tail = list(shards[t.N + lm * idx:t.N + lm * (idx + 1)])
        shards[b:b + len(tail)] = tail
        return list(shards[idx * ln:b + len(tail)])

    def repair_rows(self, bad, want):
        """cfsec_ec_repair_rows: (the N input shard indices a Reconstruct decodes from with `bad`
        lost, [rows over them, one bytes object of N per wanted shard index])."""
        N = self.CodeMode.N
        b = (ctypes.c_int * max(len(bad), 1))(*bad)
        w = (ctypes.c_int * max(len(want), 1))(*want)
        ins = (ctypes.c_int * N)()
        rows = (ctypes.c_uint8 * max(N * len(want), 1))()
        _lib.check(self._L.cfsec_ec_repair_rows(self._h, b, len(bad), w, len(want), ins, rows))
        return [ins[i] for i in range(N)], [bytes(rows[r * N:(r + 1) * N]) for r in range(len(want))]

    def matvec_batch(self, rows, ptrs, shard_size: int, nstripes: int, stream=None):
        """cfsec_ec_matvec_batch: outputs = rows x inputs on device memory; ptrs (addresses) per
        stripe: the N inputs, then one output per row."""
        from ._shards import stream_ptr
        coef = b"".join(rows)
        arr = ptrs if isinstance(ptrs, ctypes.Array) else (ctypes.c_void_p * len(ptrs))(*ptrs)
        _lib.check(self._L.cfsec_ec_matvec_batch(self._h, coef, len(rows), arr, int(shard_size), int(nstripes),
                                                 stream_ptr(stream, device=self._engine.device)))

    def shards_in_idc(self, idx: int):
        out = (ctypes.c_int * 64)()
        cnt = ctypes.c_int(0)
        _lib.check(self._L.cfsec_ec_shards_in_idc(self._h, idx, out, 64, ctypes.byref(cnt)))
        return [out[i] for i in range(cnt.value)]


def NewEncoder(cfg: Config, device: int = -1) -> Encoder:
    """ec.NewEncoder (encoder.go:78-112)."""
    if not isinstance(cfg.CodeMode, Tactic) or not cfg.CodeMode.IsValid():
        raise ErrInvalidCodeMode("ErrInvalidCodeMode")
    return Encoder(cfg, device)


@dataclass
class BufferSizes:
    """ec.BufferSizes (buf.go:52-59)."""

    ShardSize: int = 0
    DataSize: int = 0
    ECDataSize: int = 0
    ECSize: int = 0
    From: int = 0
    To: int = 0


def GetBufferSizes(dataSize: int, tactic: Tactic) -> BufferSizes:
    """ec.GetBufferSizes (buf.go:146-152 via newBuffer :67-133)."""
    frm, to = 0, dataSize
    if dataSize <= 0 or to < frm or frm < 0 or frm > dataSize or to < 0 or to > dataSize:
        raise ErrShortData("ErrShortData")
    if tactic.N <= 0:
        raise ErrInvalidCodeMode("ErrInvalidCodeMode")
    shard = (dataSize + tactic.N - 1) // tactic.N
    shard = max(shard, tactic.MinShardSize)
    return BufferSizes(shard, dataSize, shard * tactic.N, shard * (tactic.N + tactic.M + tactic.L), frm, to)
