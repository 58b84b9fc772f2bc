"""Distributed stripe repair across the GPUs of one node (BASELINE config 5).

Reference: blobnode repairs a batch of bids serially -- download the surviving shards over
HTTP, `encoder.Reconstruct(blobShards, badIdx)`, `encoder.Verify` -- in
blobstore/blobnode/work_shard_recover.go:690-771.  Here the surviving shards of a repair batch
already sit in HBM on the GPUs that own them and the only exchange is over xGMI through RCCL
(torch.distributed "nccl" backend).

Ownership: shard i of every bid lives on rank `i % world`.  Rank r holds `local`, a uint8
tensor [nbids, n_owned(r), S] with its shards in index order.

Two exchange strategies, both followed by one fused reconstruct launch per rank:

* "columns" (default): rank r rebuilds byte columns [c_r, c_r + L_r) of every erased shard of
  every bid.  One all_to_all_single sends each survivor's column slice to the rank that decodes
  it (a rank receives n_surv * S / world bytes per bid, not n_surv * S), and a second one
  returns each rebuilt slice to the erased shard's owner.
* "allgather": all_gather of every needed survivor (every rank receives all of them); the owner
  of each erased shard rebuilds it whole.  Moves world/2x more bytes; kept for comparison.

Only the first k surviving shards in index order are needed: the reference decodes from exactly
those (KRS/reedsolomon.go:1453-1465), so the exchange ships only them.

LRC modes (an ec.Encoder, e.g. EC16P20L2): the erased set may hold local parities too; the
survivors are the first N present *global* shards (lrcencoder.go:156-160 reconstructs the global
stripe first) and every erased shard -- data, global or local parity -- is one row over them
(cfsec_ec_repair_rows; a local parity through its AZ's local engine over the rebuilt AZ), so the
decode stays one launch (cfsec_ec_matvec_batch) and the exchange is unchanged.  For a consistent
stripe this equals the reference's global-then-local Reconstruct; the reference's local pass
would read the AZ's stored shards, which this exchange does not ship.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, List

import torch
import torch.distributed as dist


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


@dataclass
class RepairPlan:
    k: int
    total: int
    erased: List[int]
    survivors: List[int]  # first k present, index order

    @staticmethod
    def make(k: int, total: int, erased, nglobal: int = None) -> "RepairPlan":
        """nglobal: the survivors come from shards [0, nglobal) (LRC: the global stripe)."""
        er = sorted(set(int(e) for e in erased))
        surv = [i for i in range(total if nglobal is None else nglobal) if i not in er][:k]
        if len(surv) < k:
            from ._lib import ErrTooFewShards
            raise ErrTooFewShards("ErrTooFewShards")
        return RepairPlan(k, total, er, surv)


# ---------------------------------------------------------------- exchange ("columns")
def gather_columns(local: torch.Tensor, plan: RepairPlan, rank: int, world: int, group=None):
    """all_to_all_single: rank r receives columns [c_r, c_r+L_r) of every needed survivor of
    every bid.  Returns (recv, layout) with recv viewed per source rank as
    [nbids, n_needed_from_src, L_r] blocks, concatenated in source-rank order; layout[i] =
    (byte offset of survivor i's row for bid 0, row stride between bids)."""
    nb, S = local.shape[0], local.shape[2]
    cols = column_split(S, world)
    mine = owned(rank, plan.total, world)
    need_from = [[i for i in owned(j, plan.total, world) if i in plan.survivors] for j in range(world)]
    # send: for each destination r, my needed survivors' column slice [c_r, c_r+L_r)
    sel = [mine.index(i) for i in need_from[rank]]
    sends, send_sizes = [], []
    for r in range(world):
        c, L = cols[r]
        blk = local[:, sel, c:c + L].contiguous() if sel and L else local.new_empty(0)
        sends.append(blk.reshape(-1))
        send_sizes.append(blk.numel())
    L_me = cols[rank][1]
    recv_sizes = [nb * len(need_from[j]) * L_me for j in range(world)]
    sendbuf = torch.cat(sends) if sends else local.new_empty(0)
    recv = local.new_empty(sum(recv_sizes))
    dist.all_to_all_single(recv, sendbuf, recv_sizes, send_sizes, group=group)
    layout, off = {}, 0
    for j in range(world):
        for p, i in enumerate(need_from[j]):
            layout[i] = (off + p * L_me, len(need_from[j]) * L_me)
        off += recv_sizes[j]
    return recv, layout


def scatter_columns(rebuilt: torch.Tensor, plan: RepairPlan, rank: int, world: int, S: int, group=None):
    """Inverse exchange: rebuilt [nbids, n_erased, L_rank] column slices go to each erased shard's
    owner.  Returns [nbids, n_erased_owned(rank), S] with the whole rebuilt rows this rank owns
    (erased shards in index order)."""
    nb = rebuilt.shape[0]
    cols = column_split(S, world)
    mine_er = [e for e in plan.erased if owner(e, world) == rank]
    sends, send_sizes = [], []
    for o in range(world):
        idx = [q for q, e in enumerate(plan.erased) if owner(e, world) == o]
        blk = rebuilt[:, idx, :].contiguous() if idx else rebuilt.new_empty(0)
        sends.append(blk.reshape(-1))
        send_sizes.append(blk.numel())
    recv_sizes = [nb * len(mine_er) * cols[r][1] for r in range(world)]
    recv = rebuilt.new_empty(sum(recv_sizes))
    dist.all_to_all_single(recv, torch.cat(sends), recv_sizes, send_sizes, group=group)
    out = rebuilt.new_empty((nb, len(mine_er), S))
    off = 0
    for r in range(world):
        c, L = cols[r]
        if recv_sizes[r]:
            out[:, :, c:c + L] = recv[off:off + recv_sizes[r]].view(nb, len(mine_er), L)
        off += recv_sizes[r]
    return out


# ---------------------------------------------------------------- exchange ("allgather")
def gather_all(local: torch.Tensor, plan: RepairPlan, rank: int, world: int, group=None):
    """all_gather of every rank's needed survivors (padded to the largest count).  Returns
    (buf [world, nbids, maxn, S], layout) with layout[i] = (src rank, position)."""
    need_from = [[i for i in owned(j, plan.total, world) if i in plan.survivors] for j in range(world)]
    maxn = max(len(x) for x in need_from)
    mine = owned(rank, plan.total, world)
    nb, S = local.shape[0], local.shape[2]
    mine_blk = local.new_zeros((nb, maxn, S))
    sel = [mine.index(i) for i in need_from[rank]]
    if sel:
        mine_blk[:, :len(sel)] = local[:, sel]
    buf = local.new_empty((world, nb, maxn, S))
    dist.all_gather_into_tensor(buf.view(-1), mine_blk.view(-1), group=group)
    layout = {i: (j, p) for j in range(world) for p, i in enumerate(need_from[j])}
    return buf, layout


# ---------------------------------------------------------------- end to end (GPU)
def repair_batch(enc, local: torch.Tensor, erased, rank: int, world: int, strategy: str = "columns",
                 group=None, stream=None) -> torch.Tensor:
    """Rebuild `erased` shards of every bid of a batch whose shards are spread over `world` GPUs.

    enc: reedsolomon.ReedSolomon for (k, total-k), or an ec.Encoder (RS or LRC code mode), on this
    rank's device.  Returns the rebuilt rows this rank owns, [nbids, n_erased_owned(rank), S],
    erased shards in index order."""
    if hasattr(enc, "repair_rows"):  # ec.Encoder
        t = enc.CodeMode
        plan = RepairPlan.make(t.N, t.N + t.M + t.L, erased, nglobal=t.N + t.M)
    else:
        plan = RepairPlan.make(enc.data_shards, enc.total_shards, erased)
    nb, S = local.shape[0], local.shape[2]
    er = plan.erased
    if strategy == "columns":
        recv, layout = gather_columns(local, plan, rank, world, group)
        L = column_split(S, world)[rank][1]
        rebuilt = local.new_empty((nb, len(er), L))
        if L:
            _decode(enc, plan, nb, L, lambda i, b: recv.data_ptr() + layout[i][0] + b * layout[i][1],
                    lambda e, b: rebuilt.data_ptr() + (b * len(er) + er.index(e)) * L, stream)
        return scatter_columns(rebuilt, plan, rank, world, S, group)
    if strategy == "allgather":
        buf, layout = gather_all(local, plan, rank, world, group)
        mine_er = [e for e in er if owner(e, world) == rank]
        out = local.new_empty((nb, len(mine_er), S))
        if mine_er:
            maxn = buf.shape[2]
            # every erased row is rebuilt (the decode must not treat any as a survivor); the rows
            # other ranks own land in a scratch row
            scratch = local.new_empty((nb, S))

            def dst(e, b):
                if e in mine_er:
                    return out.data_ptr() + (b * len(mine_er) + mine_er.index(e)) * S
                return scratch.data_ptr() + b * S

            _decode(enc, plan, nb, S,
                    lambda i, b: buf.data_ptr() + ((layout[i][0] * nb + b) * maxn + layout[i][1]) * S,
                    dst, stream)
        return out
    raise ValueError(strategy)


def _decode(enc, plan: RepairPlan, nb: int, L: int, src: Callable, dst: Callable, stream):
    """One fused reconstruct launch over all bids: a full shard-pointer table per bid with the
    survivors at their exchange addresses and the erased rows at their output slots.  Present
    rows past the first k survivors are never read; they reuse a survivor's address.  With an
    ec.Encoder: the erased shards' rows over the survivors, one product launch."""
    if hasattr(enc, "repair_rows"):
        ins, rows = enc.repair_rows(plan.erased, plan.erased)
        assert ins == plan.survivors, (ins, plan.survivors)
        ptrs = []
        for b in range(nb):
            ptrs += [src(i, b) for i in ins]
            ptrs += [dst(e, b) for e in plan.erased]
        enc.matvec_batch(rows, ptrs, L, nb, stream=stream)
        return
    ptrs = []
    for b in range(nb):
        for i in range(plan.total):
            if i in plan.erased:
                ptrs.append(dst(i, b))
            elif i in plan.survivors:
                ptrs.append(src(i, b))
            else:
                ptrs.append(src(plan.survivors[0], b))
    enc.reconstruct_batch(ptrs, L, nb, plan.erased, stream=stream)
