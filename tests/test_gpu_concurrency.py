"""Concurrent and synchronous-wait forms of the scattered C5 repair (round 5).

Round 4's false ErrVerify (What's weak #1) came from the bit-sliced kernels ending with
an LDS-DMA prefetch in flight: the next workgroup placed on the CU -- another launch's, run at the
same time from another stream or process -- could have its freshly prefetched rows overwritten
(gf_bs16.hip bs_drain_exit; tools/r5_stale_dma_probe.py).  These tests run the scattered layout
(blobnode's per-vuid buffers, work_shard_recover.go:711-716) the ways that overlap launches -- two
streams at once, each call with its own flag row -- and the synchronous calls under both wait modes
(cfsec_set_sync_poll), with the rebuilt shards' checksums (work_shard_recover.go:335-342) against the
ec oracle's repair and zlib.
"""
import random
import zlib

import numpy as np
import pytest

from chubaofs_amd import _lib, codemode as cm
from oracle.ec_oracle import ECOracle, Slice

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

MODE = cm.EC16P20L2


def gen_bytes(seed, size):
    return np.random.default_rng(seed).integers(0, 256, size, dtype=np.uint8)


def enc_new():
    from chubaofs_amd import ec
    return ec.NewEncoder(ec.Config(CodeMode=cm.GetTactic(MODE), EnableVerify=False), device=0)


def oracle_repair(shards, bad):
    """work_shard_recover.go:751-760 -- Reconstruct then Verify -- restated by the ec oracle."""
    orc = ECOracle.from_tactic(cm.GetTactic(MODE))
    work = [Slice.of(s.copy()) for s in shards]
    st = orc.repair(work, list(bad), verify=True)
    return st, [w.view().copy() for w in work]


def scattered_tasklet(enc, nb, S, seed, corrupt=(), repair=True):
    """nb bids of C5's pattern {0, 1, 16, 17} (bids in `corrupt`: a compared global parity flipped),
    every shard at its own shuffled address of one pool; returns (pool, views, bads, want).  want:
    the ec oracle's repair of each bid, or (repair=False, for the large case) its status -- ErrVerify
    for the corrupted bids -- and the codeword, whose rows 0, 1, 16, 17 the repair rebuilds from
    uncorrupted rows (2..15, 18, 19) either way."""
    t = cm.GetTactic(MODE)
    n = t.N + t.M + t.L
    rnd = random.Random(seed)
    slot = S + 512
    pool = torch.zeros(nb * n * slot + 4096, dtype=torch.uint8, device="cuda")
    perm = list(range(nb * n))
    rnd.shuffle(perm)
    views, bads, want = [], [], []
    for b in range(nb):
        good = [gen_bytes(seed * 1000 + b * 64 + i, S) for i in range(t.N)] + \
               [np.zeros(S, np.uint8) for _ in range(t.M + t.L)]
        ref = [Slice.of(x) for x in good]
        assert ECOracle.from_tactic(t).encode(ref) == 0
        good = [r.view().copy() for r in ref]
        bad = [0, 1, 16, 17]
        if b in corrupt:
            good[20 + b % 10][rnd.randrange(S)] ^= 0x5A
        if repair:
            want.append(oracle_repair([g.copy() for g in good], bad))
        else:
            want.append((_lib.ErrVerify.status if b in corrupt else 0, good))
        row = []
        for i in range(n):
            o = perm[b * n + i] * slot + 16 * rnd.randrange(16)
            v = pool[o:o + S]
            v.copy_(torch.from_numpy(good[i] if i not in bad else np.zeros(S, np.uint8)))
            row.append(v)
        views.append(row)
        bads.append(bad)
    return pool, views, bads, want


@pytest.mark.parametrize("poll", [1, 0])
def test_scattered_tasklet_checksums_under_both_waits(poll):
    """Synchronous ReconstructBatch with checksums over a scattered C5 tasklet (44 bids: the device
    table route), with the call ending by the polled marker word (1) or hipStreamSynchronize (0):
    the Verify statuses, every shard and the rebuilt shards' words are those of the ec oracle and
    zlib -- the words and flags read right after the wait are complete."""
    lib = _lib.lib()
    prev = lib.cfsec_set_sync_poll(poll)
    try:
        enc = enc_new()
        S = 4096 + 2048
        pool, views, bads, want = scattered_tasklet(enc, 44, S, 11 + poll, corrupt=(3, 17, 40))
        st, crcs = enc.ReconstructBatch(views, bads, crcs=True)
        assert st == [w[0] for w in want]
        assert {w[0] for w in want} == {0, _lib.ErrVerify.status}
        n = len(views[0])
        for b, (exp, shards) in enumerate(want):
            for i in range(n):
                assert np.array_equal(views[b][i].cpu().numpy(), shards[i]), (b, i)
                w = zlib.crc32(shards[i].tobytes()) if exp == 0 and i in bads[b] else 0
                assert crcs[b][i] == w, (poll, b, i, hex(crcs[b][i]), hex(w))
    finally:
        lib.cfsec_set_sync_poll(prev)


def test_scattered_tasklets_two_streams_overlapping():
    """Two scattered C5 tasklets (64 bids x 262,144 B, erased {0, 1, 16, 17}) repaired again and again
    on two streams at once -- their bit-sliced launches overlap on the GPU, and neither blocks the
    host on the other's (the device tables are a polled ring) -- each call with its own flag row:
    exactly the corrupted bids are flagged in every call, the others in none, and the rebuilt rows
    equal the ec oracle's."""
    enc = enc_new()
    S, nb, iters = 262144, 64, 200
    sets = []
    for k in range(2):
        pool, views, bads, want = scattered_tasklet(enc, nb, S, 70 + k, corrupt=(5 + k, 33), repair=False)
        flags = torch.zeros((iters, nb), dtype=torch.int32, device="cuda")
        sets.append((pool, views, bads, want, flags, torch.cuda.Stream()))
    # marshalled once, so the host enqueues faster than the kernels run and the streams overlap
    import ctypes
    from chubaofs_amd._shards import BatchMarshal
    n = len(sets[0][1][0])
    bad = (ctypes.c_int * (4 * nb))(*([0, 1, 16, 17] * nb))
    off = (ctypes.c_int * (nb + 1))(*range(0, 4 * nb + 1, 4))
    stv = (ctypes.c_int * nb)()
    bms = [BatchMarshal(views, n) for _, views, _, _, _, _ in sets]
    torch.cuda.synchronize()
    for it in range(iters):
        for (pool, views, bads, want, flags, s), bm in zip(sets, bms):
            _lib.check(enc._L.cfsec_ec_reconstruct_batch_async(enc._h, bm.arr, n, nb, bad, off, 1, stv,
                                                               flags[it].data_ptr(), None, s.cuda_stream))
            assert list(stv) == [0] * nb
    torch.cuda.synchronize()
    for k, (pool, views, bads, want, flags, s) in enumerate(sets):
        exp = np.array([int(w[0] != 0) for w in want], np.int32)
        assert set(np.nonzero(exp)[0]) == {5 + k, 33}
        fl = (flags.cpu().numpy() != 0).astype(np.int32)
        bad_calls = [i for i in range(iters) if not np.array_equal(fl[i], exp)]
        assert not bad_calls, (k, bad_calls[:5], [np.nonzero(fl[i] != exp)[0].tolist() for i in bad_calls[:5]])
        for b, (_, shards) in enumerate(want):
            for i in bads[b]:
                assert np.array_equal(views[b][i].cpu().numpy(), shards[i]), (k, b, i)
