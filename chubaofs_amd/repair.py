"""Distributed stripe repair across the GPUs of one node (BASELINE config 5).

Reference: blobnode repairs a tasklet bid by bid -- download the surviving shards over HTTP, then
per bid `encoder.Reconstruct(blobShards, badIdx)` followed by `encoder.Verify(blobShards)`, failing
the bid with errBidCanNotRecover / errEcVerifyFailed (blobstore/blobnode/work_shard_recover.go:
706-771).  Here the shards of a tasklet already sit in HBM on the GPUs that own them and the only
exchange is over xGMI through RCCL (torch.distributed "nccl" backend).

Ownership: shard i of every bid lives on rank `i % world`.  Rank r holds `local`, a uint8 tensor
[nbids, n_owned(r), S] with its shards in index order (the bad ones' rows included: they are the
buffers the rebuilt bytes go to, exactly blobnode's `getShardBuf` of a bad shard).

Every step of the reference's per-bid repair is byte-column local -- GF(2^8) products act on each
byte position on its own, a Verify is false when any column mismatches, and every other status
(checkShards, ErrTooFewShards, the LRC local passes) depends only on the lengths and the bad sets --
so the default "columns" strategy cuts the shard length into one byte range per rank:

  1. all_to_all_single: every shard a bid's Reconstruct or Verify reads (every shard that is not bad
     in every bid) sends its column slice [c_r, c_r + L_r) to rank r != its owner -- (shards read) *
     S / world bytes per rank and bid, not (shards read) * S; a rank's own shards stay in place;
  2. rank r runs the reference's repair on its columns: cfsec_ec_reconstruct_batch_async with Verify
     (one fused Reconstruct + Verify pass per bid on the GPU; LRC bids with a bad local shard take the
     global then the AZ-local passes) over a shard table pointing into `local` and the receive
     buffer, per-bid planning status + per-bid Verify flag;
  3. all_reduce(MAX) of [status, flag] per bid: a bid fails when its columns fail anywhere;
  4. all_to_all_single returns each rebuilt slice to the bad shard's owner, which writes it into its
     `local` rows (its own columns were rebuilt there in step 2).

The per-bid result is what cfsec_ec_reconstruct_batch returns on one GPU for the whole bid:
ErrVerify where Verify is false, the Reconstruct error, or OK.  With crcs=True the rebuilt shards'
crc32.ChecksumIEEE (blobnode's ShardCrc32 of a repaired shard, work_shard_recover.go:335-342) are
combined from the column slices' checksums (cfsec_crc32_shift: x^(8 * bytes after the slice)).

"allgather" (kept for comparison): all_gather of every shard read; every rank then repairs every bid
whole (world x the decode work, world/2 x the exchange bytes of "columns").
"""
from __future__ import annotations

import ctypes
import functools
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np
import torch
import torch.distributed as dist

from . import _lib

SHARD_DTYPE = np.dtype([("data", "<u8"), ("len", "<u8"), ("cap", "<u8")])  # cfsec_shard


def owner(i: int, world: int) -> int:
    return i % world


def owned(rank: int, total: int, world: int) -> List[int]:
    return [i for i in range(total) if owner(i, world) == rank]


def column_split(S: int, world: int, align: int = 256):
    """[(start, length)] per rank; starts are `align`-aligned, the last range takes the rest."""
    chunk = -(-S // world)
    chunk = -(-chunk // align) * align
    out = []
    for r in range(world):
        a = min(r * chunk, S)
        b = min(a + chunk, S)
        out.append((a, b - a))
    return out


@dataclass(eq=False)
class RepairPlan:
    """The shape of one tasklet repair, identical on every rank (a function of the code mode and the
    bad sets only).  Plans are cached per bad-set pattern (`make`) and must not be mutated.

    bad[b]: bid b's bad shard indices (blobnode's recoverIdxOfStripe, work_shard_recover.go:715-718).
    rebuilt: shards bad in some bid, index order -- the rows the repair returns to their owners.
    shipped: shards some bid's Reconstruct or Verify reads (present in at least one bid), index order.
    slots:   the other shards (bad in every bid): no bytes cross the exchange, a rank decodes into them.
    """

    n: int
    bad: List[List[int]]
    rebuilt: List[int]
    shipped: List[int]
    slots: List[int]
    verify: bool = True
    _c: object = field(default=None, repr=False)  # the bad sets as C arrays (_bad_arrays)

    @staticmethod
    def make(n: int, nbids: int, bad, verify: bool = True) -> "RepairPlan":
        if len(bad) and isinstance(bad[0], (list, tuple, np.ndarray)):
            if len(bad) != nbids:
                raise ValueError("one bad-index list per bid")
            key = tuple(tuple(int(i) for i in b) for b in bad)
        else:
            key = tuple(int(i) for i in bad)
        return _make_plan(n, nbids, key, bool(verify))

    def order(self, world: int) -> List[int]:
        """Row order of a rank's work buffer: the shipped shards grouped by owner rank (so each source
        rank's block is contiguous in the all_to_all), then the slots."""
        return sorted(self.shipped, key=lambda i: (owner(i, world), i)) + list(self.slots)


@functools.lru_cache(maxsize=256)
def _make_plan(n: int, nbids: int, key: tuple, verify: bool) -> RepairPlan:
    if key and isinstance(key[0], tuple):
        per = [sorted(set(b)) for b in key]
    else:
        per = [sorted(set(key))] * nbids
    for b in per:
        for i in b:
            if not 0 <= i < n:
                raise IndexError(f"bad shard index {i} out of range [0, {n})")  # the reference panics
    union = sorted(set().union(*per)) if per else []
    every = sorted(set(per[0]).intersection(*per[1:])) if per else []
    shipped = [i for i in range(n) if i not in every]
    return RepairPlan(n, per, union, shipped, every, verify)


@dataclass
class RepairResult:
    """The outcome on one rank.  The rebuilt bytes are written in place into the caller's `local`
    (blobnode's setShardBuf of each recovered shard, work_shard_recover.go:762-769); `rows` gathers the
    rows of `index` from it."""

    local: torch.Tensor = field(repr=False)
    index: List[int]              # the shards this rank owns that are bad in some bid (index order)
    status: List[int]             # per bid: cfsec status (0 OK, 10 ErrVerify, or the Reconstruct error)
    crcs: Optional[np.ndarray] = None  # [nbids, len(index)] uint32: ChecksumIEEE of rows the bid rebuilt
    stats: dict = field(default_factory=dict)
    qpos: List[int] = field(default_factory=list, repr=False)  # position of index[k] in local's rows

    @property
    def rows(self) -> torch.Tensor:
        """[nbids, len(index), S]: this rank's rebuilt shards (for a bid where a shard is not bad, its
        own bytes)."""
        if not self.qpos:
            return self.local.new_empty((self.local.shape[0], 0, self.local.shape[2]))
        return self.local[:, self.qpos]


def _shard_table(nbids: int, n: int, addr: np.ndarray, length: int):
    """A cfsec_shard array of nbids * n entries {addr, length, length} (every shard full length: the
    bad ones are named by bad_idx, as blobnode passes them)."""
    t = np.zeros(max(nbids * n, 1), SHARD_DTYPE)
    t["data"][:nbids * n] = addr.reshape(-1)
    t["len"][:nbids * n] = length
    t["cap"][:nbids * n] = length
    return t


def _bad_arrays(plan: RepairPlan):
    if plan._c is None:
        flat = [i for b in plan.bad for i in b]
        off = [0]
        for b in plan.bad:
            off.append(off[-1] + len(b))
        plan._c = (ctypes.c_int * max(len(flat), 1))(*flat), (ctypes.c_int * len(off))(*off)
    return plan._c


def _repair_call(enc, plan: RepairPlan, table: np.ndarray, nbids: int, flags: torch.Tensor,
                 words: Optional[torch.Tensor], stream) -> List[int]:
    """cfsec_ec_reconstruct_batch_async over the shard table: per-bid planning status now, Verify
    flags (and checksums) on the stream."""
    bad, off = _bad_arrays(plan)
    status = (ctypes.c_int * max(nbids, 1))()
    L = enc._L
    st = L.cfsec_ec_reconstruct_batch_async(
        enc._h, table.ctypes.data_as(_lib.P_SHARD), plan.n, nbids, bad, off, int(plan.verify), status,
        flags.data_ptr(), None if words is None else words.data_ptr(), stream)
    _lib.check(st)
    return [int(status[b]) for b in range(nbids)]


def _crc_shift(words: np.ndarray, nbytes: int) -> np.ndarray:
    w = np.ascontiguousarray(words, dtype=np.uint32).copy()
    _lib.check(_lib.lib().cfsec_crc32_shift(w.ctypes.data, w.size, int(nbytes)))
    return w


def _a2a(recv: torch.Tensor, send: torch.Tensor, rsizes, ssizes, world: int, group):
    if world == 1:
        if recv.numel():
            recv.copy_(send)
        return
    dist.all_to_all_single(recv, send, rsizes, ssizes, group=group)


def _max_reduce(t: torch.Tensor, world: int, group):
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)


class _Marks:
    """Phase marks of one repair: HIP events on the current stream (read after a synchronise), or the
    host clock for CPU tensors (the gloo tests)."""

    def __init__(self, timer, dev):
        self.timer, self.cuda = timer, dev.type == "cuda"
        self.dev, self.t = dev, {}

    def mark(self, name):
        if self.timer is None:
            return
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record(torch.cuda.current_stream(self.dev))
            self.t[name] = e
        else:
            import time
            self.t[name] = time.perf_counter()

    def finish(self):
        if self.timer is None:
            return
        if self.cuda:
            torch.cuda.synchronize(self.dev)
            d = lambda a, b: self.t[a].elapsed_time(self.t[b])
        else:
            d = lambda a, b: (self.t[b] - self.t[a]) * 1e3
        self.timer.update(exchange_ms=d("t0", "sent"), decode_ms=d("sent", "decoded"),
                          return_ms=d("decoded", "returned"), total_ms=d("t0", "returned"))


def gpu_decode(enc, plan: RepairPlan, row, L: int, flags: torch.Tensor, words: Optional[torch.Tensor],
               geom=None, addr=None) -> None:
    """Step 2 on this rank's GPU: the reference's per-bid Reconstruct + Verify over the [nbids, L] rows
    of every shard (row(i): a view with its rows contiguous; geom: (base addresses, bid strides) of
    the same rows as two uint64 arrays, which spares the views; addr: the [nbids, n] row addresses
    themselves), rebuilt rows written in place.
    flags[0] receives the per-bid planning status, flags[1] the Verify flags (on the stream), words
    the rebuilt rows' checksums."""
    nb = flags.shape[1]
    if addr is None:
        if geom is None:
            base = np.empty(plan.n, np.uint64)
            stride = np.empty(plan.n, np.uint64)
            for i in range(plan.n):
                r = row(i)
                assert r.shape == (nb, L) and (L == 0 or r.stride(1) == 1)
                base[i], stride[i] = r.data_ptr(), r.stride(0)
        else:
            base, stride = geom
        addr = base[None, :] + np.arange(nb, dtype=np.uint64)[:, None] * stride[None, :]
    status = _repair_call(enc, plan, _shard_table(nb, plan.n, addr, L), nb, flags[1], words,
                          torch.cuda.current_stream(flags.device).cuda_stream)
    if any(status):
        flags[0].copy_(torch.tensor(status, dtype=torch.int32))


def _statuses(flags: torch.Tensor, S: int) -> List[int]:
    st = flags.cpu().numpy()
    if S == 0:
        return [_lib.ErrShardNoData.status] * st.shape[1]  # checkShards on all-empty shards
    return np.where(st[0] != 0, st[0], np.where(st[1] != 0, _lib.ErrVerify.status, 0)).tolist()


# ---------------------------------------------------------------- the tasklet repair
def repair_batch(enc, local: torch.Tensor, bad, rank: int, world: int, strategy: str = "columns",
                 group=None, verify: bool = True, crcs: bool = False, timer: Optional[dict] = None,
                 decode=gpu_decode) -> RepairResult:
    """Repair a tasklet whose shards are spread over `world` GPUs (shard i on rank i % world).

    enc: ec.Encoder (RS or LRC code mode) on this rank's device.  local: [nbids, n_owned, S] uint8 on
    that device.  bad: one list of bad shard indices for every bid, or one list per bid.  Runs on
    torch's current stream.  Returns this rank's rebuilt rows (every shard it owns that is bad in some
    bid; for a bid where that shard is not bad, its own bytes), the per-bid status (identical on every
    rank), and with crcs=True the rebuilt rows' checksums.  timer: a dict that receives the exchange,
    decode and return times in ms (synchronises).  decode: step 2 (gpu_decode; the CPU tests pass the
    oracle to check the exchange and the column split around it)."""
    t = enc.CodeMode
    n = t.N + t.M + t.L
    nb, n_own, S = local.shape
    if n_own != len(range(rank, n, world)):  # owned(rank, n, world)
        raise ValueError(f"rank {rank} holds {len(range(rank, n, world))} shards per bid, local has {n_own}")
    plan = RepairPlan.make(n, nb, bad, verify)
    if strategy == "columns":
        return _repair_columns(enc, local, plan, rank, world, group, crcs, timer, decode)
    if strategy == "allgather":
        return _repair_allgather(enc, local, plan, rank, world, group, crcs, timer, decode)
    raise ValueError(strategy)


@dataclass(eq=False)
class _Columns:
    """Everything about a columns repair that follows from (plan, S, world, rank, n_owned): the
    column ranges, the exchange sizes and where every shard's columns sit on this rank -- `kind`
    (0: in place in `local`, 1: the receive buffer, 2: a slot), a byte offset into that buffer and a
    bid stride.  Cached, so a repeated pattern costs the host only the addresses of its buffers."""

    cols: list
    c_me: int
    L_me: int
    mine: List[int]
    qof: dict
    sel: List[int]
    fsend: List[int]
    frecv: List[int]
    n_slots: int
    kind: np.ndarray
    off: np.ndarray
    bstride: np.ndarray
    rows_off: np.ndarray   # [nb, n] bid b's byte offset of shard i from its buffer's base
    out_idx: List[int]
    reb_by: List[List[int]]
    rsend: List[int]
    rrecv: List[int]
    _sel_t: dict = field(default_factory=dict)

    def sel_index(self, dev) -> torch.Tensor:
        """`sel` as an index tensor on `dev`, made once per device."""
        t = self._sel_t.get(dev)
        if t is None:
            t = self._sel_t[dev] = torch.tensor(self.sel, dtype=torch.int64, device=dev)
        return t


@functools.lru_cache(maxsize=256)
def _columns(plan: RepairPlan, nb: int, S: int, world: int, rank: int) -> _Columns:
    n = plan.n
    cols = column_split(S, world)
    c_me, L_me = cols[rank]
    mine = owned(rank, n, world)
    n_own = len(mine)
    qof = {i: q for q, i in enumerate(mine)}
    # shipped shards by owner; a source's block in the receive buffer is [nb, n_from[j], L_me]
    ship_by = [[i for i in plan.shipped if owner(i, world) == j] for j in range(world)]
    sel = [qof[i] for i in ship_by[rank]]
    n_me = len(sel)
    # to rank r != rank: my shipped shards' columns [c_r, c_r + L_r) as [nb, n_me, L_r]
    fsend = [0 if r == rank else n_me * nb * cols[r][1] for r in range(world)]
    frecv = [0 if j == rank else len(ship_by[j]) * nb * L_me for j in range(world)]
    others_slots = [i for i in plan.slots if owner(i, world) != rank]
    kind = np.zeros(n, np.int64)
    off = np.zeros(n, np.uint64)
    bstride = np.zeros(n, np.uint64)
    o = 0
    for j in range(world):
        if j == rank:
            continue
        for p, i in enumerate(ship_by[j]):
            kind[i], off[i], bstride[i] = 1, o + p * L_me, len(ship_by[j]) * L_me
        o += frecv[j]
    for p, i in enumerate(others_slots):
        kind[i], off[i], bstride[i] = 2, p * L_me, len(others_slots) * L_me
    for i in mine:
        kind[i], off[i], bstride[i] = 0, qof[i] * S + c_me, n_own * S
    rows_off = off[None, :] + np.arange(nb, dtype=np.uint64)[:, None] * bstride[None, :]
    out_idx = [e for e in plan.rebuilt if owner(e, world) == rank]
    reb_by = [[e for e in plan.rebuilt if owner(e, world) == o_] for o_ in range(world)]
    rsend = [0 if o_ == rank else len(reb_by[o_]) * nb * L_me for o_ in range(world)]
    rrecv = [0 if r == rank else len(out_idx) * nb * cols[r][1] for r in range(world)]
    return _Columns(cols, c_me, L_me, mine, qof, sel, fsend, frecv, len(others_slots), kind, off, bstride,
                    rows_off, out_idx, reb_by, rsend, rrecv)


def _repair_columns(enc, local, plan: RepairPlan, rank, world, group, crcs, timer, decode) -> RepairResult:
    nb, n_own, S = local.shape
    n = plan.n
    dev = local.device
    marks = _Marks(timer, dev)
    lay = _columns(plan, nb, S, world, rank)
    cols, c_me, L_me, qof = lay.cols, lay.c_me, lay.L_me, lay.qof
    marks.mark("t0")
    # 1. forward exchange: to rank r != rank, my shipped shards' columns [c_r, c_r + L_r)
    if world > 1:
        send = local.new_empty(sum(lay.fsend))
        every = lay.sel == list(range(n_own))
        idx = None if every else lay.sel_index(dev)
        n_me, o = len(lay.sel), 0
        for r in range(world):
            if lay.fsend[r]:
                c, L = cols[r]
                dst = send[o:o + lay.fsend[r]].view(nb, n_me, L)
                if every:
                    dst.copy_(local[:, :, c:c + L])
                else:  # the shipped shards' columns gathered straight into the send block
                    torch.index_select(local[:, :, c:c + L], 1, idx, out=dst)
            o += lay.fsend[r]
        recv = local.new_empty(sum(lay.frecv))
        _a2a(recv, send, lay.frecv, lay.fsend, world, group)
        del send
    else:
        recv = local.new_empty(0)
    # where shard i's columns live on this rank: in place in `local` (mine), the receive buffer
    # (others' shipped shards, [nb, n_from, L_me] per source) or a slot (others' shards bad in every
    # bid)
    slots = local.new_empty((nb, lay.n_slots, L_me))
    bufs = (local, recv, slots)
    ptrs = np.array([t_.data_ptr() for t_ in bufs], np.uint64)

    def view(i):
        t_ = bufs[lay.kind[i]]
        return t_.view(-1).as_strided((nb, L_me), (int(lay.bstride[i]), 1), t_.storage_offset() + int(lay.off[i]))

    marks.mark("sent")
    # 2. the reference's Reconstruct + Verify of every bid, on this rank's columns
    flags = torch.zeros((2, nb), dtype=torch.int32, device=dev)  # [planning status, Verify flag]
    words = torch.zeros(nb * n, dtype=torch.int32, device=dev) if crcs else None
    if L_me:
        decode(enc, plan, view, L_me, flags, words, geom=(ptrs[lay.kind] + lay.off, lay.bstride),
               addr=ptrs[lay.kind][None, :] + lay.rows_off)
    marks.mark("decoded")
    # 3. a bid fails when its columns fail on any rank
    _max_reduce(flags, world, group)
    # 4. return exchange: the rebuilt rows' columns to their owners, [nb, n_rebuilt(owner), L_me]
    out_idx, rsend, rrecv = lay.out_idx, lay.rsend, lay.rrecv
    # entered by every rank or by none (a collective): the condition depends on the plan and S only --
    # a rank with no columns (S < world * 256) or no rebuilt rows of its own still joins with empty
    # blocks (round 5: at world 8 such a rank skipped it and the others hung)
    if world > 1 and plan.rebuilt and S:
        send = local.new_empty(sum(rsend))
        o = 0
        for o_ in range(world):
            if rsend[o_]:
                blk = send[o:o + rsend[o_]].view(nb, len(lay.reb_by[o_]), L_me)
                for p, e in enumerate(lay.reb_by[o_]):
                    blk[:, p] = view(e)
            o += rsend[o_]
        recv = local.new_empty(sum(rrecv))
        _a2a(recv, send, rrecv, rsend, world, group)
        o = 0
        for r in range(world):
            if rrecv[r]:
                c, L = cols[r]
                blk = recv[o:o + rrecv[r]].view(nb, len(out_idx), L)
                for p, e in enumerate(out_idx):
                    local[:, qof[e], c:c + L] = blk[:, p]
            o += rrecv[r]
    marks.mark("returned")
    res = RepairResult(local, out_idx, _statuses(flags, S), qpos=[qof[e] for e in out_idx])
    if crcs:
        # ChecksumIEEE(row) = XOR over ranks of ChecksumIEEE(slice_r) * x^(8 * bytes after slice_r)
        w = _crc_shift(words.cpu().numpy().view(np.uint32), S - c_me - L_me) if L_me else np.zeros(nb * n, np.uint32)
        if world > 1:
            wt = torch.from_numpy(w.view(np.int32)).to(dev)
            allw = torch.empty((world, nb * n), dtype=torch.int32, device=dev)
            dist.all_gather_into_tensor(allw.view(-1), wt, group=group)
            w = np.bitwise_xor.reduce(allw.cpu().numpy().view(np.uint32), axis=0)
        w = w.reshape(nb, n)
        res.crcs = w[:, out_idx].copy() if out_idx else np.zeros((nb, 0), np.uint32)
    res.stats = {"exchange_bytes_sent": int(sum(lay.fsend)), "exchange_bytes_received": int(sum(lay.frecv)),
                 "return_bytes_received": int(sum(rrecv)), "rows_shipped": len(plan.shipped), "columns": L_me}
    marks.finish()
    return res


def _repair_allgather(enc, local, plan: RepairPlan, rank, world, group, crcs, timer, decode) -> RepairResult:
    nb, _, S = local.shape
    n = plan.n
    dev = local.device
    marks = _Marks(timer, dev)
    mine = owned(rank, n, world)
    ship_by = [[i for i in plan.shipped if owner(i, world) == j] for j in range(world)]
    maxn = max(len(x) for x in ship_by)
    marks.mark("t0")
    blk = local.new_zeros((maxn, nb, S))
    for p, i in enumerate(ship_by[rank]):
        blk[p] = local[:, mine.index(i)]
    buf = local.new_empty((world, maxn, nb, S))
    if world > 1:
        dist.all_gather_into_tensor(buf.view(-1), blk.view(-1), group=group)
    else:
        buf[0] = blk
    del blk
    slots = local.new_empty((len(plan.slots), nb, S))
    marks.mark("sent")
    where = {i: (j, p) for j in range(world) for p, i in enumerate(ship_by[j])}

    def row(i):
        if i in where:
            return buf[where[i][0], where[i][1]]
        return slots[plan.slots.index(i)]

    flags = torch.zeros((2, nb), dtype=torch.int32, device=dev)
    words = torch.zeros(nb * n, dtype=torch.int32, device=dev) if crcs else None
    if S:
        decode(enc, plan, row, S, flags, words)
    marks.mark("decoded")
    out_idx = [e for e in plan.rebuilt if owner(e, world) == rank]
    for e in out_idx:
        local[:, mine.index(e)] = row(e)
    marks.mark("returned")
    res = RepairResult(local, out_idx, _statuses(flags, S), qpos=[mine.index(e) for e in out_idx])
    if crcs:
        w = words.cpu().numpy().view(np.uint32).reshape(nb, n)
        res.crcs = np.stack([w[:, e] for e in out_idx], axis=1) if out_idx else np.zeros((nb, 0), np.uint32)
    res.stats = {"exchange_bytes_received": int((world - 1) * maxn * nb * S), "rows_shipped": len(plan.shipped)}
    marks.finish()
    return res
