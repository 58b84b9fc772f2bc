"""Multi-rank repair exchange (chubaofs_amd/repair.py) on CPU with gloo, world_size 2 and 3.

The exchanges are pure data movement: every rank must receive exactly the column slices (or
whole rows) of the first-k survivors that it decodes, and every owner must get back exactly
the rebuilt rows of its erased shards.  The GPU decode between them is covered by
tests/test_gpu_parity.py and test_repair_gpu_single_rank below.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from chubaofs_amd import repair

K, TOTAL, NB, S = 16, 38, 3, 1000  # EC16P20L2 global stripe + 2 local, odd shard size
ERASED = [0, 1, 16, 17]


def cell(b, i, n):
    """Deterministic content of shard i of bid b (n bytes)."""
    return ((np.arange(n, dtype=np.int64) * 7 + b * 131 + i * 17) % 251).astype(np.uint8)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        plan = repair.RepairPlan.make(K, TOTAL, ERASED)
        mine = repair.owned(rank, TOTAL, world)
        local = torch.from_numpy(np.stack([np.stack([cell(b, i, S) for i in mine]) for b in range(NB)]))
        # --- columns: forward exchange
        recv, layout = repair.gather_columns(local, plan, rank, world)
        c, L = repair.column_split(S, world)[rank]
        rv = recv.numpy()
        for i in plan.survivors:
            off, stride = layout[i]
            for b in range(NB):
                got = rv[off + b * stride: off + b * stride + L]
                assert np.array_equal(got, cell(b, i, S)[c:c + L]), (rank, i, b)
        assert set(layout) == set(plan.survivors)
        # --- columns: return exchange; rank r's slice of erased e, bid b = cell(b, 1000 + e, S)[cols]
        rebuilt = torch.from_numpy(np.stack([np.stack([cell(b, 1000 + e, S)[c:c + L] for e in plan.erased])
                                             for b in range(NB)])).reshape(NB, len(plan.erased), L)
        out = repair.scatter_columns(rebuilt, plan, rank, world, S)
        mine_er = [e for e in plan.erased if repair.owner(e, world) == rank]
        assert out.shape == (NB, len(mine_er), S)
        for q, e in enumerate(mine_er):
            for b in range(NB):
                assert np.array_equal(out[b, q].numpy(), cell(b, 1000 + e, S)), (rank, e, b)
        # --- allgather
        buf, lay = repair.gather_all(local, plan, rank, world)
        for i in plan.survivors:
            j, p = lay[i]
            for b in range(NB):
                assert np.array_equal(buf[j, b, p].numpy(), cell(b, i, S))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_repair_exchanges_gloo(world):
    # mp.spawn re-raises any rank's assertion in the parent
    mp.spawn(_worker, args=(world, free_port()), nprocs=world, join=True)


def test_column_split_covers_exactly():
    for S_, w in [(1000, 2), (1000, 3), (262144, 8), (5, 8), (5592406, 8)]:
        cols = repair.column_split(S_, w)
        assert sum(L for _, L in cols) == S_
        pos = 0
        for c, L in cols:
            assert c == pos or L == 0
            pos = c + L
        assert all(c % 256 == 0 for c, L in cols if L)


def test_plan_first_k_survivors():
    p = repair.RepairPlan.make(16, 36, [0, 1, 16, 17])
    assert p.survivors == list(range(2, 16)) + [18, 19]
    from chubaofs_amd._lib import ErrTooFewShards
    with pytest.raises(ErrTooFewShards):
        repair.RepairPlan.make(12, 16, [0, 1, 2, 3, 4])


@pytest.fixture(scope="module")
def nccl_world1():
    """A world-1 RCCL process group for this module, destroyed at its end."""
    if not dist.is_initialized():
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(free_port())
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    yield
    if dist.is_initialized():
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", ["columns", "allgather"])
def test_repair_gpu_single_rank(strategy, nccl_world1):
    """End to end on one GPU (world 1, RCCL): exchange + fused decode vs the oracle."""
    from chubaofs_amd import reedsolomon
    from oracle import oracle as O
    k, m, nb, S_ = 16, 20, 4, 262144 + 7
    rng = np.random.default_rng(5)
    full = []
    for b in range(nb):
        sh = [rng.integers(0, 256, S_, dtype=np.uint8) for _ in range(k)] + [np.zeros(S_, np.uint8) for _ in range(m)]
        assert O.encode(k, m, sh) == 0
        full.append(sh)
    local = torch.from_numpy(np.stack([np.stack(sh) for sh in full])).cuda()
    enc = reedsolomon.New(k, m)
    out = repair.repair_batch(enc, local, [0, 1, 16, 17], 0, 1, strategy=strategy)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for b in range(nb):
        for q, e in enumerate([0, 1, 16, 17]):
            assert np.array_equal(got[b, q], full[b][e]), (b, e)


@pytest.mark.gpu
def test_repair_gpu_tasklet_64_bids(nccl_world1):
    """The C5 shape on one GPU: a 64-bid EC16P20 tasklet (S = 262144), erased {0, 1, 16, 17},
    exchanged over RCCL (world 1) and decoded; every rebuilt row equals the original."""
    from chubaofs_amd import reedsolomon
    k, m, nb, S_ = 16, 20, 64, 262144
    g = torch.Generator(device="cuda")
    g.manual_seed(64)
    local = torch.zeros((nb, k + m, S_), dtype=torch.uint8, device="cuda")
    local[:, :k] = torch.randint(0, 256, (nb, k, S_), generator=g, device="cuda", dtype=torch.uint8)
    enc = reedsolomon.New(k, m, device=0)
    enc.encode_batch([local[b, i].data_ptr() for b in range(nb) for i in range(k + m)], S_, nb)
    torch.cuda.synchronize()
    want = local[:, [0, 1, 16, 17]].clone()
    local[:, [0, 1, 16, 17]] = 0
    out = repair.repair_batch(enc, local, [0, 1, 16, 17], 0, 1, strategy="columns")
    torch.cuda.synchronize()
    assert torch.equal(out, want)


def test_plan_lrc_survivors_are_global():
    """LRC: the survivors are the first N present global shards, never a local parity."""
    p = repair.RepairPlan.make(16, 38, [0, 36, 3], nglobal=36)
    assert p.survivors == [i for i in range(36) if i not in (0, 3)][:16]
    assert p.erased == [0, 3, 36]
    with pytest.raises(Exception):
        repair.RepairPlan.make(6, 18, list(range(11)), nglobal=16)  # 5 global shards left < 6


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", ["columns", "allgather"])
@pytest.mark.parametrize("mode,erased", [("EC16P20L2", [0, 1, 16, 36]), ("EC16P20L2", [5, 37]),
                                         ("EC6P10L2", [0, 7, 17]), ("EC6P10L2", [16, 17])])
def test_repair_gpu_lrc(mode, erased, strategy, nccl_world1):
    """LRC repair over RCCL (world 1) with an ec.Encoder: erased data, global and local parities
    rebuilt in one product launch from the first N global survivors; every rebuilt row equals the
    shard ec.Encode produced (global + every AZ's local parity, pinned to the oracle elsewhere)."""
    from chubaofs_amd import codemode as cm, ec
    t = cm.GetTactic(getattr(cm, mode))
    enc = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=False), device=0)
    total, S_, nb = t.N + t.M + t.L, 65536 + 13, 3
    rng = np.random.default_rng(len(erased) + t.N)
    full = []
    for b in range(nb):
        sh = [rng.integers(0, 256, S_, dtype=np.uint8) for _ in range(t.N)] + \
             [np.zeros(S_, np.uint8) for _ in range(t.M + t.L)]
        enc.Encode(sh)
        full.append(sh)
    local = torch.from_numpy(np.stack([np.stack(sh) for sh in full])).cuda()
    local[:, erased] = 0
    out = repair.repair_batch(enc, local, erased, 0, 1, strategy=strategy)
    torch.cuda.synchronize()
    got = out.cpu().numpy()
    for b in range(nb):
        for q, e in enumerate(sorted(erased)):
            assert np.array_equal(got[b, q], full[b][e]), (b, e)


def _gpu_worker(rank, world, port, strategy, mode):
    """One rank of a world-N repair on the box's one GPU (gloo transport: RCCL refuses two ranks on
    one device): this rank holds the shards repair.owned() assigns it, the exchange moves the
    survivors' bytes between ranks, the decode runs on the GPU, and every rebuilt row this rank owns
    must equal the shard the encoder produced."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        if mode == "EC16P20":
            from chubaofs_amd import reedsolomon
            k, total, erased = 16, 36, [0, 1, 16, 17]
            enc = reedsolomon.New(k, total - k, device=0)
        else:
            from chubaofs_amd import codemode as cm, ec
            t = cm.GetTactic(getattr(cm, mode))
            enc = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=False), device=0)
            k, total = t.N, t.N + t.M + t.L
            erased = [0, t.N + 1, t.N + t.M + 1]  # data, global parity, local parity
        nb, S_ = 3, 65536 + 13
        g = torch.Generator(device="cuda")
        g.manual_seed(777)  # every rank builds the same stripes, keeps the rows it owns
        full = torch.zeros((nb, total, S_), dtype=torch.uint8, device="cuda")
        full[:, :k] = torch.randint(0, 256, (nb, k, S_), generator=g, device="cuda", dtype=torch.uint8)
        if mode == "EC16P20":
            enc.encode_batch([full[b, i].data_ptr() for b in range(nb) for i in range(total)], S_, nb)
        else:
            for b in range(nb):
                sh = [full[b, i] for i in range(total)]
                enc.Encode(sh)
        torch.cuda.synchronize()
        mine = repair.owned(rank, total, world)
        local = full[:, mine].clone()
        for q, i in enumerate(mine):
            if i in erased:
                local[:, q] = 0
        out = repair.repair_batch(enc, local, erased, rank, world, strategy=strategy)
        torch.cuda.synchronize()
        mine_er = [e for e in sorted(erased) if repair.owner(e, world) == rank]
        assert out.shape == (nb, len(mine_er), S_)
        for q, e in enumerate(mine_er):
            assert torch.equal(out[:, q], full[:, e]), (rank, e)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("strategy", ["columns", "allgather"])
@pytest.mark.parametrize("mode", ["EC16P20", "EC16P20L2", "EC6P10L2"])
def test_repair_gpu_multi_rank_shared_device(world, strategy, mode):
    """repair_batch at world 2 and 3 end to end on the GPU -- exchange, then the decode of every
    rank's column slice (or of the gathered rows) -- the path the 8-GPU repair runs, rehearsed with
    all ranks on the box's one GPU."""
    mp.spawn(_gpu_worker, args=(world, free_port(), strategy, mode), nprocs=world, join=True)
