"""TEST INFRASTRUCTURE: CPU restatement of blobstore/common/ec's Encoder semantics (the RS
`encoder` of encoder.go and the `lrcEncoder` of lrcencoder.go) over the RS oracle of
oracle/gf_oracle.c.  Only tests/ (and bench.py's CPU legs) import this module; the product
(chubaofs_amd/, libcfsec.so) never does.

Why a separate restatement: the GPU library fuses the reference's call sequences (an LRC
Reconstruct's global pass + per-AZ local passes, a tasklet's Reconstruct + Verify per bid, the
(M+L) x N fused LRC encode), so its LRC results must be pinned by something that follows the
reference's own sequence step by step, including its slice-header quirks:

  * Go slices are modelled as `Slice(buf, len)`: `buf` is the backing array (its size is cap),
    headers are replaced, never mutated (`shards[i] = shards[i][:0]` builds a new header), and a
    sub-slice of the shard vector (`shards[:N+M]`) writes its header changes back to the caller's
    vector, as Go's shared header array does.  `GetShardsInIdc` returns a fresh header vector
    (lrcencoder.go:236-243): header changes made through it stay local, bytes are shared.
  * fillFullShards (encoder.go:199-210): every len-0 shard gets the shard size -- its old bytes
    when cap suffices, a zeroed allocation otherwise -- and is then *not* rebuilt unless its index
    is in badIdx.
  * initBadShards (encoder.go:182-188): a listed shard with len > 0 and cap > 0 becomes len 0.
  * Reconstruct (KRS/reedsolomon.go:1407-1552): a missing shard reuses its cap when it suffices,
    else a fresh buffer (AllocAligned).
  * task.Run (util/task/task.go:43-73) runs every AZ task to completion and returns the first
    error sent; when several AZs fail the reference's pick is scheduling-dependent, this oracle
    (and libcfsec) take the lowest AZ index.

Status codes are cfsec_status values (include/cfsec.h), which equal the oracle's OR_ERR_* codes.
"""
from __future__ import annotations

import numpy as np

from oracle import oracle as O

OK = 0
ERR_TOO_FEW_SHARDS = 1      # reedsolomon.ErrTooFewShards
ERR_SHARD_NO_DATA = 2       # reedsolomon.ErrShardNoData
ERR_SHARD_SIZE = 3          # reedsolomon.ErrShardSize
ERR_VERIFY = 10             # ec.ErrVerify            encoder.go:36
ERR_INVALID_SHARDS = 11     # ec.ErrInvalidShards     encoder.go:37


class Slice:
    """A Go []byte header: backing array `buf` (cap = buf.size) and `len`."""

    __slots__ = ("buf", "len")

    def __init__(self, buf=None, length=None):
        self.buf = np.zeros(0, np.uint8) if buf is None else buf
        self.len = self.buf.size if length is None else length
        assert 0 <= self.len <= self.buf.size

    @property
    def cap(self) -> int:
        return self.buf.size

    def view(self) -> np.ndarray:
        return self.buf[:self.len]

    def resliced(self, n: int) -> "Slice":
        return Slice(self.buf, n)

    @staticmethod
    def of(arr: np.ndarray) -> "Slice":
        return Slice(np.ascontiguousarray(arr, np.uint8).copy())


def vector(arrays) -> list:
    """A [][]byte from numpy arrays (copied: the oracle never aliases the caller's data)."""
    return [Slice.of(a) for a in arrays]


def views(shards) -> list:
    return [s.view().copy() for s in shards]


# ------------------------------------------------------------------ reedsolomon.Encoder (KRS)

def _check_shards(shards, nilok):
    """checkShards / shardSize, KRS/reedsolomon.go:1314-1339."""
    size = next((s.len for s in shards if s.len != 0), 0)
    if size == 0:
        return ERR_SHARD_NO_DATA, 0
    for s in shards:
        if s.len != size and (s.len != 0 or not nilok):
            return ERR_SHARD_SIZE, 0
    return OK, size


def rs_encode(k, m, shards) -> int:
    """Encode, KRS/reedsolomon.go:609-625: parity bytes written into the parity shards' arrays."""
    if len(shards) != k + m:
        return ERR_TOO_FEW_SHARDS
    err, size = _check_shards(shards, False)
    if err:
        return err
    assert O.encode(k, m, [s.buf[:size] for s in shards]) == 0
    return OK


def rs_verify(k, m, shards):
    """Verify, KRS/reedsolomon.go:770-784 -> (ok, err)."""
    if len(shards) != k + m:
        return False, ERR_TOO_FEW_SHARDS
    err, size = _check_shards(shards, False)
    if err:
        return False, err
    err, ok = O.verify(k, m, [s.buf[:size] for s in shards])
    assert err == 0
    return ok, OK


def rs_reconstruct(k, m, shards, data_only=False) -> int:
    """reconstruct, KRS/reedsolomon.go:1407-1552 (Reconstruct / ReconstructData)."""
    total = k + m
    if len(shards) != total:
        return ERR_TOO_FEW_SHARDS
    err, size = _check_shards(shards, True)
    if err:
        return err
    present = [s.len != 0 for s in shards]
    if all(present) or (data_only and all(present[:k])):
        return OK
    if sum(present) < k:
        return ERR_TOO_FEW_SHARDS
    work, new_hdr = [], {}
    for i, s in enumerate(shards):
        if present[i]:
            work.append(s.buf[:size])
        elif i < k or not data_only:
            # :1512-1518 / :1537-1543: reuse cap, else AllocAligned
            buf = s.buf if s.cap >= size else np.zeros(size, np.uint8)
            new_hdr[i] = Slice(buf, size)
            work.append(buf[:size])
        else:
            work.append(np.zeros(size, np.uint8))  # not an output: scratch the oracle ignores
    err, filled = O.reconstruct(k, m, work, present, data_only)
    if err:
        return err
    for i, h in new_hdr.items():
        assert filled[i]
        shards[i] = h
    return OK


# ------------------------------------------------------------------ ec helpers (encoder.go)

def fill_full_shards(shards) -> None:
    """fillFullShards, encoder.go:199-210 (shardSize :190-197)."""
    size = next((s.len for s in shards if s.len != 0), 0)
    for i, s in enumerate(shards):
        if s.len == 0:
            shards[i] = s.resliced(size) if s.cap >= size else Slice(np.zeros(size, np.uint8))


def init_bad_shards(shards, bad) -> None:
    """initBadShards, encoder.go:182-188 (an index past the vector panics in Go: IndexError)."""
    for i in bad:
        s = shards[i]
        if s.len != 0 and s.cap > 0:
            shards[i] = s.resliced(0)


def _sub(shards, n, fn):
    """fn(shards[:n]) with Go's shared header array: header changes land in the caller's vector."""
    sub = shards[:n]
    out = fn(sub)
    shards[:n] = sub
    return out


def layout_by_az(N, M, L, az):
    """codemode.Tactic.GetECLayoutByAZ, codemode.go:274-291 (the local stripe of each AZ)."""
    n, m, l = N // az, M // az, L // az
    return [[a * n + i for i in range(n)] + [N + a * m + i for i in range(m)] +
            [N + M + a * l + i for i in range(l)] for a in range(az)]


class ECOracle:
    """ec.NewEncoder(Config{CodeMode, EnableVerify}) (encoder.go:78-112): the RS `encoder` when
    L == 0, else the `lrcEncoder` with localEngine = New((N+M)/AZ, L/AZ)."""

    def __init__(self, N, M, L=0, AZCount=1, EnableVerify=False):
        self.N, self.M, self.L, self.AZ, self.verify_on = N, M, L, AZCount, EnableVerify
        self.ln, self.lm = (N + M) // AZCount, (L // AZCount if L else 0)

    @classmethod
    def from_tactic(cls, t, enable_verify=False):
        return cls(t.N, t.M, t.L, t.AZCount, enable_verify)

    @property
    def lrc(self) -> bool:
        return self.L != 0

    @property
    def local_size(self) -> int:
        return (self.N + self.M + self.L) // self.AZ

    def shards_in_idc(self, shards, idx):
        """lrcencoder.go:236-243: a fresh header vector of AZ idx's local stripe."""
        return [shards[g] for g in layout_by_az(self.N, self.M, self.L, self.AZ)[idx]]

    # -- Encode --
    def encode(self, shards) -> int:
        N, M, L = self.N, self.M, self.L
        if not self.lrc:  # encoder.go:114-131
            err = rs_encode(N, M, shards)
            if err:
                return err
            if self.verify_on:
                ok, err = rs_verify(N, M, shards)
                return err if err else (OK if ok else ERR_VERIFY)
            return OK
        # lrcencoder.go:35-82
        if len(shards) != N + M + L:
            return ERR_INVALID_SHARDS
        fill_full_shards(shards)
        err = _sub(shards, N + M, lambda g: rs_encode(N, M, g))
        if err:
            return err
        if self.verify_on:
            ok, err = _sub(shards, N + M, lambda g: rs_verify(N, M, g))
            if err:
                return err
            if not ok:
                return ERR_VERIFY
        errs = []
        for a in range(self.AZ):  # task.Run: every AZ task runs
            local = self.shards_in_idc(shards, a)
            err = rs_encode(self.ln, self.lm, local)
            if not err and self.verify_on:
                ok, err = rs_verify(self.ln, self.lm, local)
                if not err and not ok:
                    err = ERR_VERIFY
            errs.append(err)
        return next((e for e in errs if e), OK)

    # -- Verify -> (ok, err) --
    def verify(self, shards):
        N, M = self.N, self.M
        if not self.lrc:  # encoder.go:133-137
            return rs_verify(N, M, shards)
        # lrcencoder.go:89-131
        if len(shards) == self.local_size:
            return rs_verify(self.ln, self.lm, shards)
        if len(shards) != N + M + self.L:
            raise ValueError("the reference indexes past the shard vector (undefined here)")
        ok, err = rs_verify(N, M, shards[:N + M])
        if not ok or err:
            return ok, err
        for a in range(self.AZ):
            ok, err = rs_verify(self.ln, self.lm, self.shards_in_idc(shards, a))
            if not ok or err:
                return ok, err
        return True, OK

    # -- Reconstruct --
    def reconstruct(self, shards, bad) -> int:
        N, M, L, AZ = self.N, self.M, self.L, self.AZ
        if not self.lrc:  # encoder.go:139-144
            init_bad_shards(shards, bad)
            return rs_reconstruct(N, M, shards)
        # lrcencoder.go:133-186
        fill_full_shards(shards)
        init_bad_shards(shards, [i for i in bad if i < N + M])
        if len(shards) == self.local_size:
            return rs_reconstruct(self.ln, self.lm, shards)
        if len(shards) != N + M + L:
            raise ValueError("the reference indexes past the shard vector (undefined here)")
        err = _sub(shards, N + M, lambda g: rs_reconstruct(N, M, g))
        if err:
            return err
        local_bad = {}  # idcIdx -> local indices (:161-172); AZ order below, see module doc
        for i in bad:
            if i >= N + M:
                idc = (i - N - M) * AZ // L
                local_bad.setdefault(idc, []).append(i - N - M - L // AZ * idc + (N + M) // AZ)
        errs = []
        for idc in sorted(local_bad):
            local = self.shards_in_idc(shards, idc)
            init_bad_shards(local, local_bad[idc])
            errs.append(rs_reconstruct(self.ln, self.lm, local))
        return next((e for e in errs if e), OK)

    # -- ReconstructData --
    def reconstruct_data(self, shards, bad) -> int:
        N, M = self.N, self.M
        if not self.lrc:  # encoder.go:146-151
            init_bad_shards(shards, bad)
            return rs_reconstruct(N, M, shards, data_only=True)
        # lrcencoder.go:188-201
        if len(shards) < N + M:
            raise ValueError("the reference slices past the shard vector (undefined here)")
        _sub(shards, N + M, fill_full_shards)
        init_bad_shards(shards, [i for i in bad if i < N + M])
        return _sub(shards, N + M, lambda g: rs_reconstruct(N, M, g, data_only=True))

    # -- the blobnode repair step (work_shard_recover.go:751-760) --
    def repair(self, shards, bad, verify=True) -> int:
        """Reconstruct(shards, bad) then, with verify, Verify(shards): cfsec_ec_reconstruct_batch's
        per-bid status (the Reconstruct error, ErrVerify when Verify is false, Verify's error)."""
        err = self.reconstruct(shards, bad)
        if err or not verify:
            return err
        ok, err = self.verify(shards)
        if err:
            return err
        return OK if ok else ERR_VERIFY
