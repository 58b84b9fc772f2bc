"""Multi-rank tasklet repair (chubaofs_amd/repair.py): shards of every bid spread over ranks, the
reference's per-bid Reconstruct + Verify (blobnode/work_shard_recover.go:706-771) run on column
slices, statuses reduced over ranks, rebuilt rows returned to their owners -- always compared with
the ec oracle's whole-bid repair (oracle/ec_oracle.py ECOracle.repair, encoder.go / lrcencoder.go
step by step), never with the GPU's own encoder.

CPU (gloo, world 2/3): the whole flow with the oracle as the per-rank decoder, which checks the
exchanges, the column split and the status / checksum reduction: an oracle repair of every rank's
column slices must equal the oracle repair of the whole bids.  GPU: the same cases with the HIP
decoder (gpu_decode) at world 1 over RCCL and at world 2/3 over gloo with every rank on the box's
one GPU, C5's shape included.
"""
import os
import socket
import types
import zlib

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from chubaofs_amd import _lib, codemode as cm, repair
from oracle.ec_oracle import ECOracle, Slice, ERR_VERIFY

OK = 0


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# ---------------------------------------------------------------- tasklets
def make_tasklet(mode, nb, S, seed, bad, corrupt=()):
    """nb consistent bids of `mode` (oracle-encoded), then `corrupt`: (bid, shard, byte) flips on
    shards that survive (what a bad survivor download would hold).  bad: one list, or one per bid.
    Returns (full [nb, n, S] uint8 with the bad rows zeroed -- what their owners hold --, bad lists)."""
    t = cm.GetTactic(mode)
    o = ECOracle.from_tactic(t)
    n = t.N + t.M + t.L
    rng = np.random.default_rng(seed)
    full = np.zeros((nb, n, S), np.uint8)
    for b in range(nb):
        sh = [Slice.of(rng.integers(0, 256, S, dtype=np.uint8)) for _ in range(t.N)] + \
             [Slice(np.zeros(S, np.uint8)) for _ in range(n - t.N)]
        assert o.encode(sh) == OK
        for i in range(n):
            full[b, i] = sh[i].view()
    per = [list(x) for x in bad] if bad and isinstance(bad[0], (list, tuple)) else [list(bad)] * nb
    for b, i, p in corrupt:
        full[b, i, p % S] ^= 0x5A
    for b in range(nb):
        for i in per[b]:
            full[b, i] = 0
    return full, per


def oracle_repair(mode, full, per):
    """ECOracle.repair of every whole bid: (status per bid, rows after the repair [nb, n, S],
    ChecksumIEEE of every rebuilt shard {(bid, shard): crc})."""
    t = cm.GetTactic(mode)
    o = ECOracle.from_tactic(t)
    nb, n, S = full.shape
    out = full.copy()
    st, crc = [], {}
    for b in range(nb):
        sh = [Slice.of(full[b, i]) for i in range(n)]
        s = o.repair(sh, per[b], verify=True)
        st.append(s)
        for i in range(n):
            if sh[i].len == S:
                out[b, i] = sh[i].view()
        if s in (OK, ERR_VERIFY):
            for i in per[b]:
                crc[(b, i)] = zlib.crc32(out[b, i].tobytes()) & 0xFFFFFFFF
    return st, out, crc


def oracle_decode(enc, plan, row, L, flags, words, geom=None, addr=None):
    """Step 2 with the oracle (CPU tests only): ECOracle.repair of every bid's column slices."""
    t = enc.CodeMode
    o = ECOracle.from_tactic(t)
    nb = flags.shape[1]
    for b in range(nb):
        sh = [Slice.of(row(i)[b].numpy()) for i in range(plan.n)]
        s = o.repair(sh, plan.bad[b], verify=plan.verify)
        if s == ERR_VERIFY:
            flags[1, b] = 1
        elif s:
            flags[0, b] = s
        for i in range(plan.n):
            if sh[i].len == L:
                row(i)[b] = torch.from_numpy(sh[i].view().copy())
        if words is not None and s in (OK, ERR_VERIFY):
            for i in plan.bad[b]:
                words[b * plan.n + i] = int(np.uint32(zlib.crc32(sh[i].view().tobytes())).view(np.int32))


def check_result(res, rank, world, mode, full, per, want_st, want_rows, want_crc, crcs=True):
    t = cm.GetTactic(mode)
    n = t.N + t.M + t.L
    nb = full.shape[0]
    assert res.status == want_st, (rank, res.status, want_st)
    union = sorted(set().union(*per))
    assert res.index == [e for e in union if repair.owner(e, world) == rank]
    got = res.rows.cpu().numpy() if res.rows.is_cuda else res.rows.numpy()
    for q, e in enumerate(res.index):
        for b in range(nb):
            if e not in per[b]:
                assert np.array_equal(got[b, q], full[b, e]), (rank, b, e, "present row changed")
            elif want_st[b] in (OK, ERR_VERIFY):
                assert np.array_equal(got[b, q], want_rows[b, e]), (rank, b, e)
            if crcs and e in per[b] and want_st[b] in (OK, ERR_VERIFY):
                assert int(res.crcs[b, q]) == want_crc[(b, e)], (rank, b, e, "checksum")
    assert n == len(repair.owned(0, n, 1))


# corrupted survivors: data, global parity, local parity; bad local parities; per-bid bad sets
CASES = {
    "EC16P20L2": dict(mode=cm.EC16P20L2, nb=5, S=4096 + 37, bad=[0, 1, 16, 17],
                      corrupt=[(1, 5, 100), (2, 20, 7), (3, 36, 4000), (4, 37, 1)]),
    "EC16P20L2_local": dict(mode=cm.EC16P20L2, nb=4, S=3000, bad=[[3, 36], [3, 36], [3], [36, 20]],
                            corrupt=[(1, 4, 9), (2, 30, 2999)]),
    "EC6P10L2": dict(mode=cm.EC6P10L2, nb=4, S=2560 + 5, bad=[0, 7, 17], corrupt=[(2, 16, 11), (3, 3, 2500)]),
    "EC12P4": dict(mode=cm.EC12P4, nb=4, S=1111, bad=[0, 1, 2, 3], corrupt=[(1, 13, 3)]),
    "EC12P4_toofew": dict(mode=cm.EC12P4, nb=3, S=999, bad=[[0, 1, 2, 3, 4], [0], []], corrupt=[(1, 15, 0)]),
}
# BASELINE configs[4] at world 8 (38 shards over 8 ranks: 5,5,5,5,5,5,4,4): C5's bad set over a
# 64-bid tasklet at a small S (8 ranks' 256-B column slices, the last one ragged), and C5's own
# S = 262,144 (32 KiB columns per rank) over fewer bids; corrupted data / global / local survivors;
# EC16P20L2_local's S = 3000 leaves ranks 6 and 7 without columns (the hang round 5 found: such a
# rank skipped the return exchange)
CASES_W8 = {
    "C5_64bids": dict(mode=cm.EC16P20L2, nb=64, S=8 * 512 + 37, bad=[0, 1, 16, 17],
                      corrupt=[(3, 5, 100), (17, 20, 4000), (40, 36, 7), (63, 37, 4132)]),
    "C5_S262144": dict(mode=cm.EC16P20L2, nb=6, S=262144, bad=[0, 1, 16, 17],
                       corrupt=[(1, 2, 32768 * 3 + 5), (4, 30, 262143)]),
    "EC16P20L2_local": CASES["EC16P20L2_local"],
}


def _cpu_worker(rank, world, port, case, strategy):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.set_num_threads(1)
        c = CASES[case] if case in CASES else CASES_W8[case]
        full, per = make_tasklet(c["mode"], c["nb"], c["S"], 11, c["bad"], c["corrupt"])
        want_st, want_rows, want_crc = oracle_repair(c["mode"], full, per)
        n = full.shape[1]
        local = torch.from_numpy(full[:, repair.owned(rank, n, world)].copy())
        enc = types.SimpleNamespace(CodeMode=cm.GetTactic(c["mode"]))
        timer = {}
        res = repair.repair_batch(enc, local, per, rank, world, strategy=strategy, crcs=True, timer=timer,
                                  decode=oracle_decode)
        check_result(res, rank, world, c["mode"], full, per, want_st, want_rows, want_crc)
        assert set(timer) == {"exchange_ms", "decode_ms", "return_ms", "total_ms"}
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("strategy", ["columns", "allgather"])
@pytest.mark.parametrize("case", sorted(CASES))
def test_repair_oracle_decoder_gloo(world, strategy, case):
    """The exchange + column split + status/checksum reduction around an oracle decoder equals the
    oracle's whole-bid repair: statuses (ErrVerify on corrupted survivors, ErrTooFewShards), rebuilt
    rows, untouched present rows, and the rebuilt rows' ChecksumIEEE combined from column slices."""
    mp.spawn(_cpu_worker, args=(world, free_port(), case, strategy), nprocs=world, join=True)


@pytest.mark.parametrize("strategy", ["columns", "allgather"])
@pytest.mark.parametrize("case", sorted(CASES_W8))
def test_repair_oracle_decoder_gloo_world8(case, strategy):
    """World 8, the node BASELINE configs[4] names: the 8-way owner map, the column split (32 KiB per
    rank at S = 262,144), both exchanges and the reductions around the oracle decoder equal the
    oracle's whole-bid repair, with corrupted survivors (ErrVerify) and bad local parities."""
    c = CASES_W8[case]
    n = cm.GetTactic(c["mode"]).N + cm.GetTactic(c["mode"]).M + cm.GetTactic(c["mode"]).L
    assert [len(repair.owned(r, n, 8)) for r in range(8)] == [5, 5, 5, 5, 5, 5, 4, 4]
    if c["S"] == 262144:
        assert [L for _, L in repair.column_split(c["S"], 8)] == [32768] * 8
    if c["S"] < 8 * 512:  # ranks 6 and 7 hold no columns: they still join both exchanges (empty blocks)
        assert [L for _, L in repair.column_split(c["S"], 8)][-2:] == [0, 0]
    mp.spawn(_cpu_worker, args=(8, free_port(), case, strategy), nprocs=8, join=True)


def test_repair_oracle_decoder_world1():
    """world 1 (no process group): the exchange degenerates to local copies."""
    for case in sorted(CASES):
        c = CASES[case]
        full, per = make_tasklet(c["mode"], c["nb"], c["S"], 3, c["bad"], c["corrupt"])
        want = oracle_repair(c["mode"], full, per)
        enc = types.SimpleNamespace(CodeMode=cm.GetTactic(c["mode"]))
        for strategy in ("columns", "allgather"):
            res = repair.repair_batch(enc, torch.from_numpy(full.copy()), per, 0, 1, strategy=strategy, crcs=True,
                                      decode=oracle_decode)
            check_result(res, 0, 1, c["mode"], full, per, *want)


def test_cached_layout_follows_the_buffers():
    """Plans and column layouts are cached per bad-set pattern, never per buffer: repeated calls on
    fresh tensors (other addresses, other bytes) each repair their own tasklet."""
    c = CASES["EC16P20L2"]
    enc = types.SimpleNamespace(CodeMode=cm.GetTactic(c["mode"]))
    assert repair.RepairPlan.make(38, 4, c["bad"]) is repair.RepairPlan.make(38, 4, list(c["bad"]))
    for seed in (5, 6, 7):
        full, per = make_tasklet(c["mode"], c["nb"], c["S"], seed, c["bad"], c["corrupt"])
        want = oracle_repair(c["mode"], full, per)
        res = repair.repair_batch(enc, torch.from_numpy(full.copy()), per, 0, 1, crcs=True, decode=oracle_decode)
        check_result(res, 0, 1, c["mode"], full, per, *want)


def test_column_split_covers_exactly():
    for S_, w in [(1000, 2), (1000, 3), (262144, 8), (5, 8), (5592406, 8)]:
        cols = repair.column_split(S_, w)
        assert sum(L for _, L in cols) == S_
        pos = 0
        for c, L in cols:
            assert c == pos or L == 0
            pos = c + L
        assert all(c % 256 == 0 for c, L in cols if L)


def test_plan_rows():
    p = repair.RepairPlan.make(38, 3, [0, 1, 16, 17])
    assert p.bad == [[0, 1, 16, 17]] * 3 and p.rebuilt == [0, 1, 16, 17] and p.slots == [0, 1, 16, 17]
    assert p.shipped == [i for i in range(38) if i not in (0, 1, 16, 17)]  # every survivor: Verify reads them
    p = repair.RepairPlan.make(38, 3, [[3, 36], [3], [20]])
    assert p.rebuilt == [3, 20, 36] and p.slots == [] and p.shipped == list(range(38))
    assert p.order(2)[:19] == [i for i in range(38) if i % 2 == 0]
    with pytest.raises(IndexError):
        repair.RepairPlan.make(16, 1, [16])
    with pytest.raises(ValueError):
        repair.RepairPlan.make(16, 2, [[0]])


def test_crc32_shift_and_combine_vs_zlib():
    """cfsec_crc32_combine / cfsec_crc32_shift (host arithmetic of the C ABI) against zlib on random
    splits: the checksum of a row is the XOR of its slices' shifted checksums."""
    L = _lib.lib()
    rng = np.random.default_rng(9)
    for n in (1, 7, 256, 4099, 262144 + 3):
        a = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for cut in {0, 1, n // 3, n - 1, n}:
            c1, c2 = zlib.crc32(a[:cut]), zlib.crc32(a[cut:])
            assert L.cfsec_crc32_combine(c1, c2, n - cut) == zlib.crc32(a)
        cuts = sorted(set([0, n] + list(rng.integers(0, n + 1, 4))))
        words = np.array([zlib.crc32(a[x:y]) for x, y in zip(cuts, cuts[1:])], np.uint32)
        acc = 0
        for q, (x, y) in enumerate(zip(cuts, cuts[1:])):
            w = words[q:q + 1].copy()
            assert L.cfsec_crc32_shift(w.ctypes.data, 1, n - y) == 0
            acc ^= int(w[0])
        assert acc == zlib.crc32(a)
    assert L.cfsec_crc32_shift(None, 0, 5) == 0 and L.cfsec_crc32_shift(None, 1, 5) == _lib.ErrInvalidArg.status


# ---------------------------------------------------------------- GPU
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


def _gpu_enc(mode):
    from chubaofs_amd import ec
    return ec.NewEncoder(ec.Config(CodeMode=cm.GetTactic(mode), EnableVerify=False), device=0)


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", ["columns", "allgather"])
@pytest.mark.parametrize("case", sorted(CASES))
def test_repair_gpu_world1(case, strategy, nccl_world1):
    """RCCL world 1, HIP decoder: statuses, rebuilt rows and checksums equal the oracle's repair."""
    c = CASES[case]
    full, per = make_tasklet(c["mode"], c["nb"], c["S"], 5, c["bad"], c["corrupt"])
    want = oracle_repair(c["mode"], full, per)
    local = torch.from_numpy(full.copy()).cuda()
    res = repair.repair_batch(_gpu_enc(c["mode"]), local, per, 0, 1, strategy=strategy, crcs=True)
    torch.cuda.synchronize()
    check_result(res, 0, 1, c["mode"], full, per, *want)


@pytest.mark.gpu
def test_repair_gpu_c5_tasklet_world1(nccl_world1):
    """C5's shape: 64 bids x S = 262,144 of EC16P20L2, bad {0, 1, 16, 17}, bids 7 and 40 with a
    corrupted survivor (a global and a local parity): those fail with ErrVerify, the rest are OK and
    equal the oracle's rebuilt rows and checksums."""
    full, per = make_tasklet(cm.EC16P20L2, 64, 262144, 64, [0, 1, 16, 17], [(7, 30, 12345), (40, 37, 262143)])
    want = oracle_repair(cm.EC16P20L2, full, per)
    assert want[0][7] == ERR_VERIFY and want[0][40] == ERR_VERIFY and want[0].count(OK) == 62
    local = torch.from_numpy(full.copy()).cuda()
    timer = {}
    res = repair.repair_batch(_gpu_enc(cm.EC16P20L2), local, per, 0, 1, crcs=True, timer=timer)
    check_result(res, 0, 1, cm.EC16P20L2, full, per, *want)
    assert timer["decode_ms"] > 0


def _gpu_worker(rank, world, port, case, strategy):
    """One rank of a world-N repair on the box's one GPU (gloo transport: RCCL refuses two ranks on
    one device): this rank holds the shards repair.owned() assigns it."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        if case == "C5":
            mode, nb, S, bad, corrupt = cm.EC16P20L2, 64, 262144, [0, 1, 16, 17], [(7, 30, 12345), (40, 37, 262143),
                                                                                 (41, 2, 0)]
        else:
            c = CASES[case] if case in CASES else CASES_W8[case]
            mode, nb, S, bad, corrupt = c["mode"], c["nb"], c["S"], c["bad"], c["corrupt"]
        full, per = make_tasklet(mode, nb, S, 17, bad, corrupt)
        want = oracle_repair(mode, full, per)
        n = full.shape[1]
        local = torch.from_numpy(full[:, repair.owned(rank, n, world)].copy()).cuda()
        res = repair.repair_batch(_gpu_enc(mode), local, per, rank, world, strategy=strategy, crcs=True)
        torch.cuda.synchronize()
        check_result(res, rank, world, mode, full, per, *want)
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("strategy", ["columns", "allgather"])
@pytest.mark.parametrize("case", sorted(CASES) + ["C5"])
def test_repair_gpu_multi_rank_shared_device(world, strategy, case):
    """repair_batch at world 2 and 3 end to end with the HIP decoder -- exchange, the Reconstruct +
    Verify of every rank's column slice (or of the gathered bids), status reduction, return exchange,
    checksum combination -- against the oracle's whole-bid repair, corrupted survivors included."""
    if case == "C5" and strategy == "allgather" and world == 3:
        pytest.skip("covered by world 2; keeps the box's host memory use small")
    mp.spawn(_gpu_worker, args=(world, free_port(), case, strategy), nprocs=world, join=True)


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["EC16P20L2", "C5_64bids"])
def test_repair_gpu_world8_shared_device(case):
    """World 8 with the HIP decoder, all eight ranks on the box's one GPU (gloo transport): the
    8-way owner map and column split with the real per-rank decode, against the oracle's repair."""
    mp.spawn(_gpu_worker, args=(8, free_port(), case, "columns"), nprocs=8, join=True)
