"""The rebuilt shards' checksums computed inside the bit-sliced repair pass (round 5).

Blobnode checksums every shard a repair rebuilds (work_shard_recover.go:335-342, ShardCrc32); the
C5 tasklet (EC16P20L2, erased {0, 1, 16, 17}) used to take a second pass over the 256 rebuilt rows.
gf_bs16.hip's CRC launches fold crc32.ChecksumIEEE of the stored rows into the repair pass itself
(batch.cpp dy16_crc_group).  Every case here compares statuses, every shard and the words with the
ec oracle's repair and zlib; CFSEC_TRACE_BATCH names which groups the repair pass checksummed, so
the routing (fused: whole 2 KiB tiles, <= 4 stored rows, 0 or 2 missing data rows; else the
separate pass) is pinned too.  The route is off by default, so these tests turn it on: mode 1 (the
Horner steps inside the network, measured slower than the separate pass) and mode 2
(round 6: each wave checksums the rows of its own tiles after its last tile).
"""
import random
import re
import zlib

import numpy as np
import pytest

from chubaofs_amd import _lib, codemode as cm
from oracle.ec_oracle import ECOracle, Slice

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

MODE = cm.EC16P20L2


def enc_new():
    from chubaofs_amd import ec
    return ec.NewEncoder(ec.Config(CodeMode=cm.GetTactic(MODE), EnableVerify=False), device=0)


def codeword(S, seed):
    t = cm.GetTactic(MODE)
    rng = np.random.default_rng(seed)
    sh = [Slice.of(rng.integers(0, 256, S, dtype=np.uint8)) for _ in range(t.N)] + \
         [Slice.of(np.zeros(S, np.uint8)) for _ in range(t.M + t.L)]
    assert ECOracle.from_tactic(t).encode(sh) == 0
    return [x.view().copy() for x in sh]


def oracle_repair(shards, bad):
    orc = ECOracle.from_tactic(cm.GetTactic(MODE))
    work = [Slice.of(s.copy()) for s in shards]
    st = orc.repair(work, list(bad), verify=True)
    return st, [w.view().copy() for w in work]


def fused_counts(err):
    return [(int(a), int(b)) for a, b in re.findall(r"repair-pass crc group tasks=(\d+) fused=(\d+)", err)]


def test_repair_pass_checksums_off_by_default(monkeypatch, capfd):
    """Without CFSEC_BS_REPAIR_CRC the rebuilt shards' checksums take the separate pass."""
    monkeypatch.setenv("CFSEC_TRACE_BATCH", "1")
    monkeypatch.delenv("CFSEC_BS_REPAIR_CRC", raising=False)
    enc = enc_new()
    t = cm.GetTactic(MODE)
    n = t.N + t.M + t.L
    S, bad = 2048, [0, 1, 16, 17]
    good = codeword(S, 5)
    views = [torch.from_numpy(x.copy() if i not in bad else np.zeros(S, np.uint8)).cuda() for i, x in enumerate(good)]
    st, crcs = enc.ReconstructBatch([views], [bad], crcs=True)
    assert st == [0] and "repair-pass crc group" not in capfd.readouterr().err
    assert [crcs[0][i] for i in bad] == [zlib.crc32(good[i].tobytes()) for i in bad]
    assert [crcs[0][i] for i in range(n) if i not in bad] == [0] * (n - len(bad))


@pytest.mark.parametrize("mode", ["1", "2"])
@pytest.mark.parametrize("layout", ["slab", "scattered"])
@pytest.mark.parametrize("bad,fused", [([0, 1, 16, 17], True), ([16, 17], True), ([5, 12, 30], True),
                                       ([3, 20], False), ([0, 1, 16, 17, 18], False)])
def test_repair_pass_checksums(mode, layout, bad, fused, monkeypatch, capfd):
    """24 bids of one erasure pattern at S = 3 x 2 KiB: one slab at a bid stride (one affine launch)
    or every shard at its own address (the device row-offset table); bids 4 and 17 carry a corrupted
    compared parity (ErrVerify; their words are 0, clear_failed_crcs).  ([3, 20]: one missing data row
    -- no mode-1 form, the separate pass; mode 2 takes it.  Five rows rebuilt -- more than the kernel's 4.)"""
    monkeypatch.setenv("CFSEC_TRACE_BATCH", "1")
    monkeypatch.setenv("CFSEC_BS_REPAIR_CRC", mode)
    fused = fused or (mode == "2" and bad == [3, 20])
    enc = enc_new()
    t = cm.GetTactic(MODE)
    n = t.N + t.M + t.L
    S, nb = 3 * 2048, 24
    rnd = random.Random(len(bad) * 7 + (layout == "slab"))
    want, srcs = [], []
    for b in range(nb):
        good = codeword(S, 1000 + b)
        if b in (4, 17):
            j = next(x for x in range(16, 36) if x not in bad and x not in (18, 19, 20, 21))
            good[j][rnd.randrange(S)] ^= 0x24
        want.append(oracle_repair(good, bad))
        srcs.append(good)
    if layout == "slab":
        buf = torch.zeros((nb, n, S), dtype=torch.uint8, device="cuda")
        views = [[buf[b, i] for i in range(n)] for b in range(nb)]
    else:
        slot = S + 512
        pool = torch.zeros(nb * n * slot + 4096, dtype=torch.uint8, device="cuda")
        perm = list(range(nb * n))
        rnd.shuffle(perm)
        views = [[pool[perm[b * n + i] * slot + 16 * rnd.randrange(8):][:S] for i in range(n)] for b in range(nb)]
    for b in range(nb):
        for i in range(n):
            views[b][i].copy_(torch.from_numpy(srcs[b][i] if i not in bad else np.zeros(S, np.uint8)))
    st, crcs = enc.ReconstructBatch(views, [bad] * nb, crcs=True)
    err = capfd.readouterr().err
    assert st == [w[0] for w in want]
    assert st[4] == _lib.ErrVerify.status and st[17] == _lib.ErrVerify.status
    for b, (exp, shards) in enumerate(want):
        for i in range(n):
            assert np.array_equal(views[b][i].cpu().numpy(), shards[i]), (b, i)
            w = zlib.crc32(shards[i].tobytes()) if exp == 0 and i in bad else 0
            assert crcs[b][i] == w, (layout, bad, b, i, hex(crcs[b][i]), hex(w))
    counts = fused_counts(err)
    if fused:
        assert counts and sum(f for _, f in counts) == nb, err
    else:
        assert sum(f for _, f in counts) == 0, err


@pytest.mark.parametrize("mode", ["1", "2"])
def test_repair_pass_checksums_c5_async_and_tail(mode, monkeypatch):
    """C5's tasklet (64 bids x 262,144 B) through the asynchronous call with device words -- every
    rebuilt shard's word equals zlib's, the Verify flags of the two corrupted bids set -- and the same
    tasklet at S = 262,144 + 48 (a row tail: the separate pass), equal words."""
    monkeypatch.setenv("CFSEC_BS_REPAIR_CRC", mode)
    enc = enc_new()
    t = cm.GetTactic(MODE)
    n = t.N + t.M + t.L
    bad = [0, 1, 16, 17]
    for S in (262144, 262144 + 48):
        nb = 64 if S == 262144 else 8
        buf = torch.zeros((nb, n, S), dtype=torch.uint8, device="cuda")
        gold = [codeword(S, 77 + b) for b in range(nb)]
        corrupt = {9: 25, 40: 37} if nb == 64 else {3: 25}
        for b, j in corrupt.items():
            gold[b] = [x.copy() for x in gold[b]]
            gold[b][j][12345] ^= 0x42
        for b in range(nb):
            for i in range(n):
                if i not in bad:
                    buf[b, i].copy_(torch.from_numpy(gold[b][i]))
        views = [[buf[b, i] for i in range(n)] for b in range(nb)]
        flags = torch.zeros(nb, dtype=torch.int32, device="cuda")
        words = torch.full((nb * n,), -1, dtype=torch.int32, device="cuda")
        st = enc.ReconstructBatchAsync(views, [bad] * nb, flags=flags, crcs=words)
        torch.cuda.synchronize()
        assert st == [0] * nb
        fl = flags.cpu().numpy()
        assert set(np.nonzero(fl)[0]) == set(corrupt), fl
        got = words.cpu().numpy().astype(np.uint32).reshape(nb, n)
        for b in range(nb):
            rebuilt = buf[b].cpu().numpy()
            for i in range(n):
                if i in bad:
                    assert np.array_equal(rebuilt[i], gold[b][i]) or b in corrupt, (S, b, i)
                    assert got[b][i] == zlib.crc32(rebuilt[i].tobytes()), (S, b, i)
                else:
                    assert got[b][i] == 0, (S, b, i)
