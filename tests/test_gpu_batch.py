"""Heterogeneous stripe batches (cfsec_rs_*_stripes, cfsec_ec_reconstruct_batch) on the GPU.

The reference repairs a blobnode tasklet bid by bid (blobnode/work_shard_recover.go:708-771): each
bid has its own shard size and its own broken shards, and each runs encoder.Reconstruct then
encoder.Verify.  Here one call does the whole batch; every bid must come out exactly as the two
reference calls leave it -- bytes from the oracle's two-pass reconstruct (KRS/reedsolomon.go:
1407-1552, restated in oracle/gf_oracle.c) and the Verify verdict from the oracle's Verify -- on
consistent stripes and on stripes whose unused parity was corrupted (Verify false).  The bid
sizes are worker_for_test.go's {1024, 2048, 0, 512, 23, 65, 12} (:79-83) with its genMockBytes
data (:62-69), plus larger and odd sizes.
"""
import random

import numpy as np
import pytest

from chubaofs_amd import _lib, codemode as cm
from oracle import oracle as O
from oracle.ec_oracle import ECOracle, Slice

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

MOCK_SIZES = [1024, 2048, 0, 512, 23, 65, 12]  # worker_for_test.go:79-83
RS_MODES = [(6, 6), (12, 4), (15, 12), (12, 9), (16, 20), (10, 4), (3, 3), (40, 4)]  # k = 40: compared rows over > 32 inputs;
# (15, 12), (12, 9): the lookup-product kernels (gf_lut.hpp)


def gen_mock_bytes(letter, size):
    """worker_for_test.go:62-69"""
    return ((letter + np.arange(size)) & 0xFF).astype(np.uint8)


def codeword(k, m, size, bid):
    sh = [gen_mock_bytes(bid + i, size) for i in range(k)] + [np.zeros(size, np.uint8) for _ in range(m)]
    assert size == 0 or O.encode(k, m, sh) == 0
    return sh


def reference_repair(k, m, shards, bad, verify=True):
    """Reconstruct then Verify with the oracle, as the reference's two calls; returns (status,
    shards after)."""
    n = k + m
    work = [s.copy() for s in shards]
    present = [i not in bad for i in range(n)]
    S = len(shards[0])
    if S == 0:
        return _lib.ErrShardNoData.status, work
    if sum(present) < k:
        return _lib.ErrTooFewShards.status, work
    if not all(present):
        err, _ = O.reconstruct(k, m, work, present)
        if err:
            return err, work
    if verify:
        err, ok = O.verify(k, m, work)
        if err:
            return err, work
        if not ok:
            return _lib.ErrVerify.status, work
    return 0, work


def to_mem(shards, memory):
    if memory == "device":
        return [torch.from_numpy(np.ascontiguousarray(s)).cuda() for s in shards]
    if memory == "pinned":
        out = []
        for s in shards:
            p = _lib.pinned_empty(s.size)
            p[:] = s
            out.append(p)
        return out
    return [s.copy() for s in shards]


def host(x):
    return x.cpu().numpy() if hasattr(x, "cpu") else np.asarray(x)


def mark_missing(stripe, bad, memory):
    for i in bad:
        stripe[i] = stripe[i][:0]  # len 0 = missing; the call gives it a fresh buffer


@pytest.mark.parametrize("memory", ["host", "pinned", "device"])
@pytest.mark.parametrize("k,m", RS_MODES)
def test_reconstruct_stripes_mock_bids(k, m, memory):
    from chubaofs_amd import reedsolomon
    enc = reedsolomon.New(k, m, device=0)
    r = random.Random(k * 100 + m)
    sizes = MOCK_SIZES + [174763, 4096, 1, 100003]
    stripes, want, bads = [], [], []
    for b, size in enumerate(sizes):
        good = codeword(k, m, size, b + 1)
        nbad = r.randint(0, m)
        bad = sorted(r.sample(range(k + m), nbad))
        src = [s.copy() for s in good]
        corrupt = b % 3 == 2 and nbad < m and size > 0  # an unused present parity goes bad
        if corrupt:
            spare = [i for i in range(k + m) if i not in bad][k:]  # present beyond the first k
            j = spare[-1]
            src[j][size // 2] ^= 0x5A
        stripes.append(to_mem(src, memory))
        mark_missing(stripes[-1], bad, memory)
        bads.append(bad)
        want.append(reference_repair(k, m, src, bad))
    status = enc.ReconstructStripes(stripes, verify=True)
    for b, (st, shards) in enumerate(want):
        assert status[b] == st, (b, sizes[b], bads[b], status[b], st)
        if st in (0, _lib.ErrVerify.status):
            got = [host(x) for x in stripes[b]]
            for i in range(k + m):
                assert np.array_equal(got[i], shards[i]), (b, sizes[b], bads[b], i)


@pytest.mark.parametrize("memory", ["host", "device"])
@pytest.mark.parametrize("verify", [True, False])
def test_reconstruct_stripes_16_20_dyadic_repair(memory, verify):
    """The 16 + 20 code (EC16P20, EC16P20L2's global stripe) with up to 4 data shards missing takes
    repair_dy16 when it verifies (decode rows for the missing data, then all 20 parity rows through
    the 16x16 dyadic block): every split of the erasures between data and parity, corrupted parity
    outside and inside the first 16 present shards, odd sizes, against the oracle's two passes."""
    from chubaofs_amd import reedsolomon
    k, m = 16, 20
    enc = reedsolomon.New(k, m, device=0)
    r = random.Random(1620 + verify)
    stripes, want, cases = [], [], []
    b = 0
    for nd in range(5):
        for npar in (0, 1, 2, 4, 9):
            for corrupt in ("none", "spare", "input"):
                size = r.choice([1, 23, 4096, 4097, 65536 + 5, 262144])
                good = codeword(k, m, size, b)
                bad = sorted(r.sample(range(k), nd) + r.sample(range(k, k + m), npar))
                src = [x.copy() for x in good]
                present = [i for i in range(k + m) if i not in bad]
                if corrupt == "spare" and len(present) > k:
                    src[present[-1]][size // 2] ^= 0x5A  # verified, not an input
                if corrupt == "input" and nd > 0:
                    src[present[k - 1]][0] ^= 0x33  # a parity shard among the first 16 present
                stripes.append(to_mem(src, memory))
                mark_missing(stripes[-1], bad, memory)
                want.append(reference_repair(k, m, src, bad, verify=verify))
                cases.append((nd, npar, corrupt, size, bad))
                b += 1
    status = enc.ReconstructStripes(stripes, verify=verify)
    for i, (st, shards) in enumerate(want):
        assert status[i] == st, (cases[i], status[i], st)
        got = [host(x) for x in stripes[i]]
        for j in range(k + m):
            assert np.array_equal(got[j], shards[j]), (cases[i], j)


@pytest.mark.parametrize("memory", ["host", "device"])
def test_reconstruct_stripes_many_patterns_and_launch_splits(memory):
    """70 stripes (more than one launch's 32 length slots), 9 erasure patterns, varied sizes."""
    from chubaofs_amd import reedsolomon
    k, m = 12, 4
    enc = reedsolomon.New(k, m, device=0)
    r = random.Random(5)
    patterns = [sorted(r.sample(range(16), r.randint(1, 4))) for _ in range(9)]
    stripes, want = [], []
    for b in range(70):
        size = r.choice([37, 4096, 4097, 65536 + 3, 300001])
        good = codeword(k, m, size, b)
        bad = patterns[b % len(patterns)]
        stripes.append(to_mem(good, memory))
        mark_missing(stripes[-1], bad, memory)
        want.append(good)
    assert enc.ReconstructStripes(stripes) == [0] * 70
    for b in range(70):
        for i in range(16):
            assert np.array_equal(host(stripes[b][i]), want[b][i]), (b, i)


def test_reconstruct_stripes_pageable_two_lanes():
    """A pageable host batch larger than one staging lane (256 MiB): chunks alternate over the two
    lanes of the device."""
    from chubaofs_amd import reedsolomon
    k, m, S = 12, 4, 1 << 20
    enc = reedsolomon.New(k, m, device=0)
    rng = np.random.default_rng(3)
    base = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
    assert O.encode(k, m, base) == 0
    stripes, want = [], []
    for b in range(24):  # 24 x 16 MiB = 384 MiB of staging
        good = [np.roll(x, b) for x in base[:k]] + [np.zeros(S, np.uint8) for _ in range(m)]
        assert enc.EncodeStripes([good]) == [0]
        want.append([x.copy() for x in good])
        bad = [b % 16, (b + 5) % 16]
        mark_missing(good, bad, "host")
        stripes.append(good)
    assert enc.ReconstructStripes(stripes) == [0] * 24
    for b in range(24):
        for i in range(16):
            assert np.array_equal(stripes[b][i], want[b][i]), (b, i)
    assert np.array_equal(want[0][k], base[k])  # the GPU encode of stripe 0 equals the oracle's


@pytest.mark.parametrize("memory", ["host", "device"])
def test_encode_and_verify_stripes(memory):
    from chubaofs_amd import reedsolomon
    k, m = 6, 6
    enc = reedsolomon.New(k, m, device=0)
    sizes = [1, 15, 16, 17, 2048, 174763, 0, 5]
    stripes, want = [], []
    for b, size in enumerate(sizes):
        good = codeword(k, m, size, b) if size else [np.zeros(0, np.uint8)] * (k + m)
        src = [x.copy() for x in good[:k]] + [np.full(size, 0xEE, np.uint8) for _ in range(m)]
        stripes.append(to_mem(src, memory))
        want.append(good)
    st = enc.EncodeStripes(stripes)
    assert st == [0 if s else _lib.ErrShardNoData.status for s in sizes]
    for b, size in enumerate(sizes):
        for i in range(k + m):
            assert np.array_equal(host(stripes[b][i]), want[b][i]), (b, i)
    stripes[3][k + 2][5] ^= 1
    vs = enc.VerifyStripes(stripes)
    assert vs[3] == _lib.ErrVerify.status and vs[6] == _lib.ErrShardNoData.status
    assert all(v == 0 for i, v in enumerate(vs) if i not in (3, 6))


def test_set_devices():
    from chubaofs_amd import reedsolomon
    enc = reedsolomon.New(12, 4, device=0)
    enc.SetDevices([0])
    with pytest.raises(_lib.ErrInvalidArg):
        enc.SetDevices([0, 0])
    with pytest.raises(_lib.ErrDevice):
        enc.SetDevices([0, 4096])
    good = codeword(12, 4, 4096, 1)
    st = [x.copy() for x in good]
    mark_missing(st, [0, 13], "host")
    assert enc.ReconstructStripes([st]) == [0]
    assert all(np.array_equal(a, b) for a, b in zip(st, good))


# ------------------------------------------------------------------ ec.Encoder batches

def ec_new(mode):
    from chubaofs_amd import ec
    return ec.NewEncoder(ec.Config(CodeMode=cm.GetTactic(mode), EnableVerify=False))


def ec_full_codeword(enc, t, size, bid):
    shards = [gen_mock_bytes(bid + i, size) for i in range(t.N)] + \
             [np.zeros(size, np.uint8) for _ in range(t.M + t.L)]
    enc.Encode(shards)
    return shards


def sequential(enc, shards, bad, verify=True):
    """The reference loop body (work_shard_recover.go:751-760): Reconstruct then Verify, restated on
    the CPU by the ec oracle (oracle/ec_oracle.py: lrcencoder.go / encoder.go over the RS oracle) --
    never by the GPU's own single-call path."""
    orc = ECOracle.from_tactic(enc.CodeMode)
    work = [Slice() if s.size == 0 else Slice.of(s) for s in shards]
    st = orc.repair(work, list(bad), verify=verify)
    return st, [w.view().copy() for w in work]


@pytest.mark.parametrize("memory", ["host", "device"])
@pytest.mark.parametrize("mode", [cm.EC6P6, cm.EC12P4, cm.EC15P12, cm.EC6P10L2, cm.EC16P20L2, cm.EC4P4L2, cm.EC6P3L3])
def test_ec_reconstruct_batch_matches_repair_loop(mode, memory):
    """cfsec_ec_reconstruct_batch over a tasklet == the per-bid Reconstruct + Verify of the ec oracle,
    global stripes, with corrupted bids."""
    t = cm.GetTactic(mode)
    enc = ec_new(mode)
    total = t.N + t.M + t.L
    r = random.Random(mode)
    bids, bads, want = [], [], []
    for b, size in enumerate([1024, 2048, 512, 23, 65, 12, 262144, 4097]):
        good = ec_full_codeword(enc, t, size, b + 1)
        nbad = r.randint(1, t.M)
        bad = sorted(r.sample(range(total), nbad))
        src = [x.copy() for x in good]
        if b % 3 == 1:  # corrupt a surviving parity (global or local) outside the bad set
            cand = [i for i in range(t.N, total) if i not in bad]
            src[cand[-1]][size // 3] ^= 0x81
        want.append(sequential(enc, src, bad))
        work = to_mem(src, memory)
        for i in bad:
            if memory == "device":
                work[i].zero_()
            else:
                work[i][:] = 0  # a broken shard's buffer, still full length (work_shard_recover.go)
        bids.append(work)
        bads.append(bad)
    status = enc.ReconstructBatch(bids, bads)
    for b, (st, shards) in enumerate(want):
        assert status[b] == st, (b, bads[b], status[b], st)
        if st in (0, _lib.ErrVerify.status):
            for i in range(total):
                assert np.array_equal(host(bids[b][i]), shards[i]), (b, bads[b], i)


@pytest.mark.parametrize("memory", ["host", "device"])
@pytest.mark.parametrize("mode", [cm.EC6P10L2, cm.EC16P20L2])
def test_ec_reconstruct_batch_local_verify_in_global_pass(mode, memory):
    """Bids with no bad local shard have their local Verify done in the global pass (the local
    parities are compared there as rows over the data): every outcome equals the per-bid
    Reconstruct + Verify calls -- a corrupted local parity of either AZ, a corrupted global parity,
    a clean bid, and bids whose bad set holds a local parity (rebuilt by the local pass) mixed into
    one tasklet; C5's pattern {0, 1, 16, 17} for EC16P20L2 runs the 16x16-dyadic repair kernel."""
    t = cm.GetTactic(mode)
    enc = ec_new(mode)
    total = t.N + t.M + t.L
    base = [0, 1, 16, 17] if mode == cm.EC16P20L2 else [0, 7]
    cases = [("clean", base), ("local0", base), ("local1", base), ("global", base),
             ("clean", base + [total - 1]), ("local0", base + [total - 1]), ("data", base)]
    bids, bads, want = [], [], []
    for b, (corrupt, bad) in enumerate(cases):
        size = [262144, 4097, 65, 2048, 23, 1024, 777][b]
        good = ec_full_codeword(enc, t, size, 40 + b)
        src = [x.copy() for x in good]
        at = (size * (b + 1)) // 8
        if corrupt == "local0":
            src[t.N + t.M][at] ^= 0x5A
        elif corrupt == "local1":
            src[t.N + t.M + t.L - 1][at] ^= 0x21
        elif corrupt == "global":
            src[t.N + t.M - 1][at] ^= 0x80
        elif corrupt == "data":
            src[t.N - 1][at] ^= 0x01  # an input: the rebuilt rows follow it, some check fails
        want.append(sequential(enc, src, bad))
        work = to_mem(src, memory)
        for i in bad:
            if memory == "device":
                work[i].zero_()
            else:
                work[i][:] = 0
        bids.append(work)
        bads.append(bad)
    status = enc.ReconstructBatch(bids, bads)
    for b, (st, shards) in enumerate(want):
        exp = 0 if cases[b][0] == "clean" else _lib.ErrVerify.status
        assert st == exp, (b, cases[b], st)
        assert status[b] == st, (b, cases[b], status[b], st)
        for i in range(total):
            assert np.array_equal(host(bids[b][i]), shards[i]), (b, cases[b], i)


@pytest.mark.parametrize("mode", [cm.EC6P10L2, cm.EC16P20L2])
def test_ec_reconstruct_batch_local_stripes(mode):
    """AZ-local repair (lrcencoder.go:147-152): a batch of local stripes (n = local stripe size)."""
    t = cm.GetTactic(mode)
    enc = ec_new(mode)
    ln = (t.N + t.M + t.L) // t.AZCount
    bids, bads, want = [], [], []
    for b, size in enumerate([699051, 1024, 23]):
        good = ec_full_codeword(enc, t, size, b)
        az = b % t.AZCount
        idx, _, _ = t.LocalStripeInAZ(az)
        local = [good[i].copy() for i in idx]
        bad = [b % ln]
        want.append(sequential(enc, local, bad))
        work = [x.copy() for x in local]
        work[bad[0]][:] = 0
        bids.append(work)
        bads.append(bad)
    assert enc.ReconstructBatch(bids, bads) == [w[0] for w in want]
    for b, (_, shards) in enumerate(want):
        for i in range(ln):
            assert np.array_equal(bids[b][i], shards[i]), (b, i)


@pytest.mark.parametrize("memory", ["host", "device"])
@pytest.mark.parametrize("mode", [cm.EC6P6, cm.EC12P4, cm.EC6P10L2, cm.EC16P20L2, cm.EC6P3L3, cm.EC4P4L2])
@pytest.mark.parametrize("verify", [False, True])
def test_ec_encode_batch_matches_encode(mode, memory, verify):
    """cfsec_ec_encode_batch (access puts batched, LRC fused) == per-stripe Encode of the ec oracle
    (global + every AZ's local parity, lrcencoder.go:35-82), including stripes with missing parity
    or local shards (fillFullShards), a missing data shard, and a local parity of another length
    (global parity written, ErrShardSize)."""
    from chubaofs_amd import ec
    t = cm.GetTactic(mode)
    enc = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=verify))
    orc = ECOracle.from_tactic(t, enable_verify=verify)
    total = t.N + t.M + t.L
    stripes, want, exp = [], [], []
    for b, size in enumerate([1, 23, 2048, 4097, 699051, 65536, 777, 1000]):
        data = [gen_mock_bytes(b * 7 + i, size) for i in range(t.N)]
        src = data + [np.full(size, 0x5A, np.uint8) for _ in range(total - t.N)]
        if b == 6:
            src[total - 1] = src[total - 1][:0]  # a missing (local) parity: filled, then encoded
            src[t.N] = src[t.N][:0]
        if b == 7 and t.L:
            src[total - 1] = np.zeros(size + 1, np.uint8)  # a local shard of another length
        elif b == 7:
            src[1] = src[1][:0]  # RS: a missing data shard is an error (checkShards)
        ref = [Slice() if x.size == 0 else Slice.of(x) for x in src]
        exp.append(orc.encode(ref))
        want.append([r.view().copy() for r in ref])
        stripes.append(to_mem([x.copy() for x in src], memory))
    assert enc.EncodeBatch(stripes) == exp
    for b in range(len(stripes)):
        for i in range(total):
            assert np.array_equal(host(stripes[b][i]), want[b][i]), (b, i)


# ------------------------------------------------------------------ asynchronous batches

@pytest.mark.parametrize("mode", [cm.EC12P4, cm.EC16P20L2, cm.EC6P10L2, cm.EC15P12])
def test_ec_reconstruct_batch_async_matches_oracle(mode):
    """cfsec_ec_reconstruct_batch_async: planning status at return, Verify verdicts in the device
    flags once the stream has passed; bytes as the ec oracle's Reconstruct + Verify.  Two tasklets
    back to back on one stream without a sync in between (the second reuses no workspace the first
    still holds)."""
    t = cm.GetTactic(mode)
    enc = ec_new(mode)
    total = t.N + t.M + t.L
    r = random.Random(mode * 3)
    stream = torch.cuda.Stream()
    rounds = []
    for rnd in range(2):
        bids, bads, want = [], [], []
        for b, size in enumerate([262144, 4097, 23, 65536, 1, 2048]):
            good = ec_full_codeword(enc, t, size, 9 * rnd + b)
            bad = sorted(r.sample(range(total), r.randint(1, t.M)))
            src = [x.copy() for x in good]
            if b % 2 == 1:
                cand = [i for i in range(t.N, total) if i not in bad]
                src[cand[r.randrange(len(cand))]][size // 2] ^= 0x3C
            want.append(sequential(enc, src, bad))
            work = to_mem(src, "device")
            for i in bad:
                work[i].zero_()
            bids.append(work)
            bads.append(bad)
        torch.cuda.synchronize()
        flags = torch.zeros(len(bids), dtype=torch.int32, device="cuda")
        with torch.cuda.stream(stream):
            st = enc.ReconstructBatchAsync(bids, bads, flags=flags)
        rounds.append((bids, want, st, flags))
    stream.synchronize()
    for bids, want, st, flags in rounds:
        fl = flags.cpu().numpy()
        for b, (exp, shards) in enumerate(want):
            got = ErrVerify if (st[b] == 0 and fl[b]) else st[b]
            assert got == exp, (cm.Name(mode), b, st[b], fl[b], exp)
            if exp in (0, ErrVerify):
                for i in range(total):
                    assert np.array_equal(host(bids[b][i]), shards[i]), (b, i)


ErrVerify = _lib.ErrVerify.status


@pytest.mark.parametrize("mode", [cm.EC12P4, cm.EC6P10L2, cm.EC16P20L2])
def test_ec_encode_batch_async_matches_oracle(mode):
    from chubaofs_amd import ec
    t = cm.GetTactic(mode)
    enc = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=True), device=0)
    orc = ECOracle.from_tactic(t, enable_verify=True)
    total = t.N + t.M + t.L
    stripes, want, exp = [], [], []
    for b, size in enumerate([1, 4097, 699051, 0]):
        src = [gen_mock_bytes(b * 5 + i, size) for i in range(t.N)] + \
              [np.full(size, 0x11, np.uint8) for _ in range(total - t.N)]
        ref = [Slice() if x.size == 0 else Slice.of(x) for x in src]
        exp.append(orc.encode(ref))
        want.append([x.view().copy() for x in ref])
        stripes.append(to_mem(src, "device"))
    torch.cuda.synchronize()
    flags = torch.zeros(len(stripes), dtype=torch.int32, device="cuda")
    st = enc.EncodeBatchAsync(stripes, flags=flags)
    torch.cuda.synchronize()
    assert st == exp and not flags.any().item()
    for b in range(len(stripes)):
        for i in range(total):
            assert np.array_equal(host(stripes[b][i]), want[b][i]), (b, i)


def test_async_rejects_host_memory_and_missing_flags():
    enc = ec_new(cm.EC12P4)
    t = enc.CodeMode
    good = ec_full_codeword(enc, t, 4096, 1)
    with pytest.raises(TypeError):
        enc.ReconstructBatchAsync([[x.copy() for x in good]], [[0]])
    dev = [to_mem(good, "device")]
    with pytest.raises(_lib.ErrInvalidArg):
        enc.ReconstructBatchAsync(dev, [[0]], flags=None, verify=True)


# ------------------------------------------------------------------ multi-device split, rehearsed

def _trace_split(err):
    """{device index: [items]} from the library's CFSEC_TRACE_BATCH lines."""
    out = {}
    for line in err.splitlines():
        if line.startswith("cfsec batch: device index"):
            head, items = line.split(", items")
            d = int(head.split("device index")[1].split()[0])
            out.setdefault(d, []).append([int(x) for x in items.split()])
    return out


@pytest.mark.parametrize("memory", ["host", "pinned"])
def test_two_device_split_rehearsed(memory, monkeypatch, capfd):
    """The device-set path (run_stripes: one host thread, stream pair and staging per device, stripes
    split by cfsec_batch_partition) with two contexts on device 0 (CFSEC_DEVICE_REHEARSAL): bytes
    equal the oracle's two-pass reconstruct + Verify, and the split is the partition's."""
    from chubaofs_amd import reedsolomon
    monkeypatch.setenv("CFSEC_DEVICE_REHEARSAL", "1")
    monkeypatch.setenv("CFSEC_TRACE_BATCH", "1")
    k, m = 12, 4
    enc = reedsolomon.New(k, m, device=0)
    enc.SetDevices([0, 0])
    sizes = [4096, 300001, 23, 1 << 20, 65537, 777, 200000, 5]
    bad = [0, 5, 13]
    stripes, want = [], []
    for b, size in enumerate(sizes):
        good = codeword(k, m, size, b + 3)
        src = [x.copy() for x in good]
        if b == 2:
            src[15][size // 2] ^= 0x40  # a compared parity: Verify false
        want.append(reference_repair(k, m, src, bad))
        stripes.append(to_mem(src, memory))
        mark_missing(stripes[-1], bad, memory)
    capfd.readouterr()
    status = enc.ReconstructStripes(stripes, verify=True)
    err = capfd.readouterr().err
    for b, (st, shards) in enumerate(want):
        assert status[b] == st, (b, status[b], st)
        for i in range(k + m):
            assert np.array_equal(host(stripes[b][i]), shards[i]), (b, i)
    # every stripe moves (k inputs + 3 rebuilt + 1 compared parity) rows of its size
    expect = _lib.batch_partition([s * (k + 4) for s in sizes], 2)
    split = _trace_split(err)
    assert set(split) == {0, 1}, err
    got = {d: sorted(i for call in v for i in call) for d, v in split.items()}
    assert got == {d: [i for i, x in enumerate(expect) if x == d] for d in (0, 1)}, (got, expect)


def test_two_device_lrc_tasklet_rehearsed(monkeypatch, capfd):
    """An LRC tasklet (global pass, then AZ-local passes of the bids with a bad local shard) over two
    rehearsed device contexts: every pass of a bid stays on one device, results equal the ec oracle."""
    monkeypatch.setenv("CFSEC_DEVICE_REHEARSAL", "1")
    monkeypatch.setenv("CFSEC_TRACE_BATCH", "1")
    t = cm.GetTactic(cm.EC6P10L2)
    enc = ec_new(cm.EC6P10L2)
    enc.SetDevices([0, 0])
    total = t.N + t.M + t.L
    bids, bads, want = [], [], []
    for b, size in enumerate([4097, 65536, 23, 262144, 1000, 12]):
        good = ec_full_codeword(enc, t, size, 70 + b)
        bad = [0, total - 1] if b % 2 else [2, 9]
        src = [x.copy() for x in good]
        if b == 3:
            src[t.N + t.M][7] ^= 1
        want.append(sequential(enc, src, bad))
        work = to_mem(src, "pinned" if b % 3 == 0 else "host")
        for i in bad:
            work[i][:] = 0
        bids.append(work)
        bads.append(bad)
    capfd.readouterr()
    status = enc.ReconstructBatch(bids, bads)
    err = capfd.readouterr().err
    for b, (st, shards) in enumerate(want):
        assert status[b] == st, (b, status[b], st)
        for i in range(total):
            assert np.array_equal(host(bids[b][i]), shards[i]), (b, i)
    split = _trace_split(err)
    assert set(split) == {0, 1}, err
    seen = {}
    for d, calls in split.items():
        for call in calls:
            for it in call:
                assert seen.setdefault(it, d) == d, ("a bid's passes split over devices", it)


# ------------------------------------------------------------------ checksums from the batch calls

def crc_of(a):
    return O.crc32_ieee(np.ascontiguousarray(a)) if a.size else 0


@pytest.mark.parametrize("memory", ["host", "pinned", "device"])
@pytest.mark.parametrize("mode", [cm.EC6P6, cm.EC12P4, cm.EC6P10L2, cm.EC16P20L2])
def test_ec_encode_batch_crc(mode, memory):
    """cfsec_ec_encode_batch_crc: the ec oracle's Encode, then crc32.ChecksumIEEE of every shard
    (access/stream_put.go:249-253) -- zlib-equal words from the GPU; a failed stripe's words are 0."""
    from chubaofs_amd import ec
    t = cm.GetTactic(mode)
    enc = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=True), device=0)
    orc = ECOracle.from_tactic(t, enable_verify=True)
    total = t.N + t.M + t.L
    stripes, want, exp = [], [], []
    for b, size in enumerate([1, 23, 4096, 4097, 262144, 0, 65537]):
        src = [gen_mock_bytes(b * 11 + i, size) for i in range(t.N)] + \
              [np.full(size, 0x42, np.uint8) for _ in range(total - t.N)]
        ref = [Slice() if x.size == 0 else Slice.of(x) for x in src]
        exp.append(orc.encode(ref))
        want.append([x.view().copy() for x in ref])
        stripes.append(to_mem(src, memory))
    st, crcs = enc.EncodeBatch(stripes, crcs=True)
    assert st == exp
    for b in range(len(stripes)):
        for i in range(total):
            assert np.array_equal(host(stripes[b][i]), want[b][i]), (b, i)
            w = crc_of(want[b][i]) if exp[b] == 0 else 0
            assert crcs[b][i] == w, (b, i, hex(crcs[b][i]), hex(w))
    import zlib
    assert crcs[3][0] == zlib.crc32(want[3][0].tobytes())


@pytest.mark.parametrize("memory", ["host", "pinned", "device"])
@pytest.mark.parametrize("mode", [cm.EC12P4, cm.EC16P20L2, cm.EC6P10L2, cm.EC6P6])
def test_ec_reconstruct_batch_crc(mode, memory):
    """cfsec_ec_reconstruct_batch_crc: the rebuilt shards' checksums (blobnode's ShardCrc32 of each
    repaired shard, work_shard_recover.go:335-342) -- global, data and local parity alike -- 0 for
    the shards not rebuilt and for bids whose status is not OK; C5's pattern at S = 262,144."""
    t = cm.GetTactic(mode)
    enc = ec_new(mode)
    total = t.N + t.M + t.L
    r = random.Random(mode + 17)
    bids, bads, want = [], [], []
    for b, size in enumerate([262144, 4097, 23, 65536, 1, 2048, 777]):
        good = ec_full_codeword(enc, t, size, 30 + b)
        if mode == cm.EC16P20L2 and b == 0:
            bad = [0, 1, 16, 17]
        elif t.L and b == 1:
            bad = [2, total - 1]
        else:
            bad = sorted(r.sample(range(total), r.randint(1, t.M)))
        src = [x.copy() for x in good]
        if b == 5:
            cand = [i for i in range(t.N, total) if i not in bad]
            src[cand[0]][size // 2] ^= 0x18
        want.append(sequential(enc, src, bad))
        work = to_mem(src, memory)
        for i in bad:
            if memory == "device":
                work[i].zero_()
            else:
                work[i][:] = 0
        bids.append(work)
        bads.append(bad)
    st, crcs = enc.ReconstructBatch(bids, bads, crcs=True)
    for b, (exp, shards) in enumerate(want):
        assert st[b] == exp, (b, st[b], exp)
        for i in range(total):
            assert np.array_equal(host(bids[b][i]), shards[i]), (b, i)
            w = crc_of(shards[i]) if exp == 0 and i in bads[b] else 0
            assert crcs[b][i] == w, (cm.Name(mode), b, bads[b], i, hex(crcs[b][i]), hex(w))


def test_ec_reconstruct_batch_async_crc():
    t = cm.GetTactic(cm.EC16P20L2)
    enc = ec_new(cm.EC16P20L2)
    total = t.N + t.M + t.L
    bids, bads, want = [], [], []
    for b, size in enumerate([262144, 4096, 5]):
        good = ec_full_codeword(enc, t, size, 90 + b)
        bad = [0, 1, 16, 17] if b != 1 else [3, total - 2]
        want.append(sequential(enc, good, bad))
        work = to_mem(good, "device")
        for i in bad:
            work[i].zero_()
        bids.append(work)
        bads.append(bad)
    flags = torch.zeros(len(bids), dtype=torch.int32, device="cuda")
    crcs = torch.full((len(bids) * total,), -1, dtype=torch.int32, device="cuda")
    st = enc.ReconstructBatchAsync(bids, bads, flags=flags, crcs=crcs)
    torch.cuda.synchronize()
    assert st == [0] * len(bids) and not flags.any().item()
    got = crcs.cpu().numpy().astype(np.uint32).reshape(len(bids), total)
    for b, (_, shards) in enumerate(want):
        for i in range(total):
            assert got[b][i] == (crc_of(shards[i]) if i in bads[b] else 0), (b, i)


@pytest.mark.parametrize("size", [1, 17, 4095, 4097, 65539, 699051])
def test_lrc_fused_encode_crc_ragged(size, monkeypatch, capfd):
    """EC6P10L2's fused LRC encode + all 18 checksums (C4's put, stream_put.go:249-253; round 6: the
    bit-sliced network with checksums from its bit planes, gf_bs_crc.hip): 5 equal-length bids in
    device memory (one fused launch), ragged and whole-tile sizes; parity against the ec oracle's
    Encode, every word against crc32.ChecksumIEEE."""
    monkeypatch.setenv("CFSEC_TRACE_BATCH", "1")
    from chubaofs_amd import ec
    t = cm.GetTactic(cm.EC6P10L2)
    total = t.N + t.M + t.L
    enc = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=False), device=0)
    orc = ECOracle.from_tactic(t, enable_verify=False)
    stripes, want = [], []
    for b in range(5):
        src = [gen_mock_bytes(b * 13 + i, size) for i in range(t.N)] + \
              [np.full(size, 0x5A, np.uint8) for _ in range(total - t.N)]
        ref = [Slice.of(x) for x in src]
        assert orc.encode(ref) == 0
        want.append([x.view().copy() for x in ref])
        stripes.append(to_mem(src, "device"))
    capfd.readouterr()
    st, crcs = enc.EncodeBatch(stripes, crcs=True)
    assert "fused crc group k=6 m=12 tasks=5" in capfd.readouterr().err
    assert st == [0] * 5
    for b in range(5):
        for i in range(total):
            assert np.array_equal(host(stripes[b][i]), want[b][i]), (b, i)
            assert crcs[b][i] == crc_of(want[b][i]), (b, i)


@pytest.mark.parametrize("gap", [False, True])
@pytest.mark.parametrize("memory", ["host", "device"])
@pytest.mark.parametrize("mode", [cm.EC12P4, cm.EC6P6, cm.EC6P10L2])
def test_ec_batch_crc_uniform_groups(mode, memory, gap, monkeypatch, capfd):
    """The batch calls' checksums when a group holds many equal-length tasks -- the case the fused
    product + CRC launch takes (batch.cpp fused_crc_group: one task per bid, one checksum-word
    stride); with gap, a failed bid in the middle breaks the stride and the separate pass runs.
    Reconstruct: a corrupted bid fails Verify after the fused launch wrote its words (they read 0)."""
    monkeypatch.setenv("CFSEC_TRACE_BATCH", "1")
    from chubaofs_amd import ec
    t = cm.GetTactic(mode)
    total = t.N + t.M + t.L
    size = 65536
    rs = t.L == 0
    # encode
    enc = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=True), device=0)
    orc = ECOracle.from_tactic(t, enable_verify=True)
    stripes, want, exp = [], [], []
    for b in range(6):
        src = [gen_mock_bytes(b * 7 + i, size) for i in range(t.N)] + \
              [np.zeros(size, np.uint8) for _ in range(total - t.N)]
        if gap and b == 2:
            src[1] = src[1][:-1].copy()  # shard size mismatch: the bid fails before any launch
        ref = [Slice.of(x) for x in src]
        exp.append(orc.encode(ref))
        want.append([x.view().copy() for x in ref])
        stripes.append(to_mem(src, memory))
    capfd.readouterr()
    st, crcs = enc.EncodeBatch(stripes, crcs=True)
    err = capfd.readouterr().err
    assert st == exp
    assert (exp[2] != 0) == gap
    for b in range(6):
        for i in range(total):
            assert np.array_equal(host(stripes[b][i]), want[b][i]), (b, i)
            assert crcs[b][i] == (crc_of(want[b][i]) if exp[b] == 0 else 0), (b, i)
    fused = "fused crc group k=%d m=%d tasks=6" % (t.N, t.M + t.L)
    if memory == "device" and not gap:  # EC6P10L2: the 6 x (10 + 2) fused LRC encode + 18 checksums
        assert fused in err, err
    if gap:
        assert "tasks=6" not in err and "tasks=5" not in err, err
    # reconstruct: the same bad set everywhere (one plan, one group).  With a parity of slack the plan
    # also compares the survivors (Verify's rows: not a plain store, the separate pass runs) and bid 3
    # is corrupted; with exactly M erasures nothing is left to compare and the group fuses.
    enc = ec_new(mode)
    for slack in ([1, 0] if rs else [1]):
        bad = list(range(t.M - slack)) if rs else [0, total - 1]
        bids, bads, wantr = [], [], []
        for b in range(6):
            good = ec_full_codeword(enc, t, size, 50 + b)
            src = [x.copy() for x in good]
            bb = list(bad)
            if b == 3 and slack:
                src[total - 1 if rs else t.N][size // 3] ^= 0x21
            if gap and b == 1:
                bb = list(range(t.M + t.L + 1))  # too many erasures: no task for this bid
            wantr.append(sequential(enc, src, bb))
            work = to_mem(src, memory)
            for i in bb:
                if memory == "device":
                    work[i].zero_()
                else:
                    work[i][:] = 0
            bids.append(work)
            bads.append(bb)
        capfd.readouterr()
        st, crcs = enc.ReconstructBatch(bids, bads, crcs=True)
        err = capfd.readouterr().err
        assert (wantr[3][0] != 0) == bool(slack)
        for b, (e, shards) in enumerate(wantr):
            assert st[b] == e, (b, st[b], e)
            for i in range(total):
                assert np.array_equal(host(bids[b][i]), shards[i]), (b, i)
                assert crcs[b][i] == (crc_of(shards[i]) if e == 0 and i in bads[b] else 0), (b, i)
        if not slack and memory == "device" and not gap:
            assert "fused crc group k=%d m=%d tasks=6" % (t.N, t.M) in err, err
        if slack or gap:
            assert "fused crc group" not in err, err


@pytest.mark.parametrize("call", ["sync", "async"])
@pytest.mark.parametrize("mode", [cm.EC12P4, cm.EC16P20L2])
def test_verify_flags_direct_and_gathered(mode, call):
    """Verify verdicts by both routes of batch.cpp: bids 0, 2, 4 share one erasure set and 1, 3, 5
    another (each group's items are not consecutive: per-task words + the gather launch), 6 and 7 a
    third (consecutive: the kernel writes the items' words directly).  Bids 2 and 7 are corrupted.
    Asynchronous flags accumulate: bid 5's word preset to 1 stays 1 (engine.hpp AsyncOut)."""
    t = cm.GetTactic(mode)
    enc = ec_new(mode)
    total = t.N + t.M + t.L
    sets = ([[0, 5], [1, 13], [2, 3]] if mode == cm.EC12P4 else [[0, 17], [3, 20], [0, 1, 16, 17]])
    plan = [0, 1, 0, 1, 0, 1, 2, 2]
    bids, bads, want = [], [], []
    for b, p in enumerate(plan):
        size = 65536
        good = ec_full_codeword(enc, t, size, 200 + b)
        bad = list(sets[p])
        src = [x.copy() for x in good]
        if b in (2, 7):
            cand = [i for i in range(t.N, t.N + t.M) if i not in bad]
            src[cand[-1]][size // 5] ^= 0x81
        want.append(sequential(enc, src, bad))
        work = to_mem(src, "device")
        for i in bad:
            work[i].zero_()
        bids.append(work)
        bads.append(bad)
    assert want[2][0] != 0 and want[7][0] != 0
    if call == "sync":
        st = enc.ReconstructBatch(bids, bads)
        got = list(st)
    else:
        flags = torch.zeros(len(bids), dtype=torch.int32, device="cuda")
        flags[5] = 1
        torch.cuda.synchronize()
        st = enc.ReconstructBatchAsync(bids, bads, flags=flags)
        torch.cuda.synchronize()
        fl = flags.cpu().numpy()
        assert fl[5] == 1
        got = [ErrVerify if (s == 0 and fl[b] and b != 5) else s for b, s in enumerate(st)]
        assert [int(v) for v in fl] == [int(b in (2, 5, 7)) for b in range(len(bids))], fl
    for b, (exp, shards) in enumerate(want):
        assert got[b] == exp, (cm.Name(mode), call, b, got[b], exp)
        for i in range(total):
            assert np.array_equal(host(bids[b][i]), shards[i]), (b, i)


def test_async_over_32_inputs_not_supported():
    """A Verify over more than 32 inputs takes the synchronous stripe-by-stripe path, which cannot
    honour an asynchronous call's stream: the _async forms return ErrNotSupported for it (no code
    mode has more than 16 inputs; a custom 40 + 4 tactic reaches it), the synchronous call works."""
    from chubaofs_amd import ec
    from chubaofs_amd.codemode import Tactic
    t = Tactic(40, 4, 0, 1, 42, 0, 0)
    enc = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=True), device=0)
    S = 4096
    good = [gen_mock_bytes(i, S) for i in range(40)] + [np.zeros(S, np.uint8) for _ in range(4)]
    assert enc.EncodeBatch([good]) == [0]  # parity written into good
    dev = [torch.from_numpy(x.copy()).cuda() for x in good]
    flags = torch.zeros(1, dtype=torch.int32, device="cuda")
    with pytest.raises(_lib.ErrNotSupported):
        enc.EncodeBatchAsync([dev], flags=flags)
    with pytest.raises(_lib.ErrNotSupported):
        enc.ReconstructBatchAsync([dev], [[0]], flags=flags)
    st = enc.ReconstructBatch([[x.copy() for x in good]], [[0]])
    assert st == [0]


@pytest.mark.parametrize("S", [4096, 6144 + 48])
def test_ec16p20l2_scattered_encode_batch_bitsliced(S):
    """An encode batch of the 16 + 20 code whose shards each sit at their own address, more stripes
    than one argument block holds: the bit-sliced encode through a device table of row offsets (one
    launch), the rows' 48-byte tails on the pointer-table chunks -- every parity (and local) row
    against the ec oracle's Encode (lrcencoder.go / encoder.go over KRS)."""
    mode = cm.EC16P20L2
    t = cm.GetTactic(mode)
    n = t.N + t.M + t.L
    enc = ec_new(mode)
    nb = 24
    rnd = random.Random(S + 7)
    slot = S + 512
    pool = torch.full((nb * n * slot + 4096,), 0xA5, dtype=torch.uint8, device="cuda")
    perm = list(range(nb * n))
    rnd.shuffle(perm)
    views, want = [], []
    for b in range(nb):
        data = [gen_mock_bytes(900 + 31 * b + i, S) for i in range(t.N)]
        ref = [Slice.of(d) for d in data] + [Slice.of(np.zeros(S, np.uint8)) for _ in range(t.M + t.L)]
        assert ECOracle.from_tactic(t).encode(ref) == 0
        want.append([r.view().copy() for r in ref])
        row = []
        for i in range(n):
            o = perm[b * n + i] * slot + 16 * rnd.randrange(16)
            v = pool[o:o + S]
            if i < t.N:
                v.copy_(torch.from_numpy(data[i]))
            row.append(v)
        views.append(row)
    assert enc.EncodeBatch(views) == [0] * nb
    for b in range(nb):
        for i in range(n):
            assert np.array_equal(views[b][i].cpu().numpy(), want[b][i]), (mode, S, b, i)


@pytest.mark.parametrize("S", [4096, 6144 + 48])
def test_ec16p20l2_scattered_tasklet_bitsliced_repair(S):
    """C5-shaped repairs whose shards each sit at their own address (blobnode assembles a bid from
    per-vuid buffers, work_shard_recover.go:711-716): the bit-sliced repair over a table of row
    offsets (~20 bids per launch: the 24 bids of C5's pattern take 2), the dyadic kernel for the 48-byte row
    tails and for three missing data rows -- statuses and every shard against the ec oracle's
    repair loop, with corrupted compared parities, data and local rows."""
    mode = cm.EC16P20L2
    t = cm.GetTactic(mode)
    n = t.N + t.M + t.L
    enc = ec_new(mode)
    patterns = [[16, 17], [3, 20], [0, 1, 16, 17], [6, 25], [4, 11], [8, 14], [7, 13], [0, 1, 2, 16]]
    nb = 44
    rnd = random.Random(S + 1)
    slot = S + 512
    pool = torch.zeros(nb * n * slot + 4096, dtype=torch.uint8, device="cuda")
    perm = list(range(nb * n))
    rnd.shuffle(perm)
    views, bads, want = [], [], []
    for b in range(nb):
        good = ec_full_codeword(enc, t, S, 500 + b)
        bad = [0, 1, 16, 17] if b < 24 else patterns[b % len(patterns)]  # 24 of C5's pattern: 2 launches
        work = [g.copy() for g in good]
        for i in bad:
            work[i][:] = 0
        if b % 11 == 5:  # a compared global parity corrupted
            j = next(x for x in range(16, 36) if x not in bad)
            work[j][rnd.randrange(S)] ^= 0x3C
        if b % 11 == 7:  # a present data row corrupted
            j = next(x for x in range(16) if x not in bad)
            work[j][rnd.randrange(S)] ^= 0x81
        if b % 13 == 9:  # a local parity corrupted
            work[37][rnd.randrange(S)] ^= 0x11
        want.append(sequential(enc, [w.copy() for w in work], bad))
        row = []
        for i in range(n):
            o = perm[b * n + i] * slot + 16 * rnd.randrange(16)
            v = pool[o:o + S]
            v.copy_(torch.from_numpy(work[i]))
            row.append(v)
        views.append(row)
        bads.append(bad)
    status = enc.ReconstructBatch(views, bads)
    assert status == [w[0] for w in want], (status, [w[0] for w in want])
    assert {w[0] for w in want} == {0, _lib.ErrVerify.status}
    for b in range(nb):
        for i in range(n):
            assert np.array_equal(views[b][i].cpu().numpy(), want[b][1][i]), (S, b, bads[b], i)


@pytest.mark.parametrize("S", [4096, 262144 + 2048 + 48])
def test_ec16p20l2_tasklet_bitsliced_repair(S):
    """C5-shaped repairs through the bit-sliced repair kernel (gf_bs16.hip: aligned rows of one
    [bids, 38, S] buffer, pairs of bids per erasure pattern so every group is one affine run; S =
    264,240 leaves a 48-byte row tail to the dyadic kernel): nothing missing but parities ({16, 17}),
    one and two missing data rows ({3, 20}, {0, 1, 16, 17}), the same with a corrupted compared parity
    and a corrupted data row (Verify must fail), and three missing data rows (the dyadic kernel);
    the paired basis' slot cases -- one even slot ({6, 25}), even + odd in different pairs ({4, 11}),
    two even ({8, 14}), two odd ({7, 13}) -- statuses and every shard against the reference loop
    restated by the ec oracle."""
    mode = cm.EC16P20L2
    t = cm.GetTactic(mode)
    n = t.N + t.M + t.L
    enc = ec_new(mode)
    patterns = [[16, 17], [3, 20], [0, 1, 16, 17], [0, 1, 16, 17], [5, 30], [0, 1, 2, 16],
                [6, 25], [4, 11], [8, 14], [7, 13]]
    nb = 2 * len(patterns)
    buf = torch.empty((nb, n, S), dtype=torch.uint8, device="cuda")
    assert buf.data_ptr() % 16 == 0
    rnd = random.Random(S)
    bads, want = [], []
    for b in range(nb):
        good = ec_full_codeword(enc, t, S, 100 + b)
        bad = patterns[b // 2]
        work = [g.copy() for g in good]
        for i in bad:
            work[i][:] = 0
        if b in (6, 7):  # a compared global parity (bid 6) / a present data row (bid 7) corrupted
            j = 25 if b == 6 else 9
            work[j][rnd.randrange(S)] ^= 1 + rnd.randrange(255)
        if b == 9:  # a local parity corrupted
            work[37][rnd.randrange(S)] ^= 0x11
        if b == 17:  # the present partner of a missing even slot (9 beside 8) corrupted
            work[9][rnd.randrange(S)] ^= 0x5A
        want.append(sequential(enc, [w.copy() for w in work], bad))
        buf[b] = torch.from_numpy(np.stack(work))
        bads.append(bad)
    status = enc.ReconstructBatch([[buf[b, i] for i in range(n)] for b in range(nb)], bads)
    assert status == [w[0] for w in want], (status, [w[0] for w in want])
    got = buf.cpu().numpy()
    assert {w[0] for w in want} == {0, _lib.ErrVerify.status}
    for b in range(nb):  # ErrVerify bids too: the reference's Reconstruct wrote them before Verify
        for i in range(n):
            assert np.array_equal(got[b, i], want[b][1][i]), (S, b, bads[b], i)
