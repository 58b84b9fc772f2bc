"""The ec.Encoder oracle (oracle/ec_oracle.py) on the CPU, pinned to the reference's own tests
before any GPU result is compared with it:

* TestLrcEncoder (blobstore/common/ec/encoder_test.go:108-247) and TestLrcReconstruct (:249-307,
  every code mode) restated step by step on the oracle, every `require` kept as an assert;
* the golden mock stripes (tests/golden/ec_golden.json, blobnode/worker_for_test.go's bids) come
  out of the oracle's LRC Encode byte for byte;
* the slice-header quirks the module doc lists (fill-not-rebuild of a missing shard outside
  badIdx, cap reuse, the localBadIdx remap, early return of Verify) on hand-made cases.
"""
import hashlib
import json
import os
import random

import numpy as np
import pytest

from chubaofs_amd import codemode as cm
from oracle import oracle as O
from oracle.ec_oracle import (ECOracle, Slice, ERR_SHARD_SIZE, ERR_TOO_FEW_SHARDS, ERR_INVALID_SHARDS,
                              ERR_VERIFY, rs_reconstruct, vector, views)

SRC = b"Hello world"  # encoder_test.go:30
GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ec_golden.json")))


def go_split(t, data: bytes, size=None):
    """encoder.Split (KRS/reedsolomon.go:1574-1632 + lrcencoder.go:203-222) of a slice whose cap
    equals its len: N+M capped shards of ceil(len/N) bytes, data then zero padding, plus L zeroed
    local shards."""
    per = (len(data) + t.N - 1) // t.N
    flat = np.zeros(per * (t.N + t.M), np.uint8)
    flat[:len(data)] = np.frombuffer(data, np.uint8)
    return [Slice(flat[i * per:(i + 1) * per].copy()) for i in range(t.N + t.M)] + \
           [Slice(np.zeros(per, np.uint8)) for _ in range(t.L)]


def join(t, shards, n):
    return b"".join(s.view().tobytes() for s in shards[:t.N])[:n]


def test_lrc_encoder_flow_ec6p10l2():
    """encoder_test.go:108-247 on the oracle."""
    t = cm.GetTactic(cm.EC6P10L2)
    enc = ECOracle.from_tactic(t, enable_verify=True)
    shards = go_split(t, SRC)
    assert enc.encode(shards[:-1]) == ERR_INVALID_SHARDS
    assert enc.encode([]) == ERR_INVALID_SHARDS
    assert enc.encode(shards) == 0
    assert join(t, shards, len(SRC)) == SRC

    shards[0].buf[:] = 222
    assert enc.verify(shards) == (False, 0)
    assert enc.reconstruct_data(shards, [0]) == 0
    assert join(t, shards, len(SRC)) == SRC

    local = enc.shards_in_idc(shards, 0)
    for idx in range(len(local)):
        local[idx].buf[:] = 11
        assert enc.verify(shards) == (False, 0)
        assert enc.reconstruct(local, [idx]) == 0
        assert enc.verify(shards) == (True, 0)

    bad = [t.N + t.M + 1]
    shards[t.N + t.M + 1].buf[:] = 222
    assert enc.verify(shards) == (False, 0)
    for i in range(t.M):
        if i % 2 == 0:
            bad.append(i)
            if i < t.N:
                shards[i].buf[:] = 222
        else:
            bad.append(t.N + i)
            shards[t.N + i].buf[:] = 222
    assert enc.verify(shards) == (False, 0)
    assert enc.reconstruct(shards, bad) == 0
    assert enc.verify(shards) == (True, 0)
    assert join(t, shards, len(SRC)) == SRC

    shards[bad[0]] = shards[bad[0]].resliced(0)
    ok, err = enc.verify(shards)
    assert err != 0 and not ok
    assert enc.reconstruct(shards, bad) == 0
    shards[bad[-1]] = shards[len(bad) - 1].resliced(0)  # the test's own index quirk, kept
    ok, err = enc.verify(shards)
    assert err != 0 and not ok


@pytest.mark.parametrize("mode", cm.GetAllCodeModes())
def test_lrc_reconstruct_flow_all_modes(mode):
    """encoder_test.go:249-307 (testLrcReconstruct) on the oracle."""
    t = cm.GetTactic(mode)
    enc = ECOracle.from_tactic(t, enable_verify=True)
    rng = np.random.default_rng(mode)
    data = rng.integers(0, 256, (1 << 12) + int(rng.integers(0, 1 << 12)), dtype=np.uint8).tobytes()
    shards = go_split(t, data)
    assert enc.encode(shards) == 0
    origin = views(shards)
    bads = []
    for b in range(t.N + t.M, t.N + t.M + t.L):
        bads.append(b)
        for i in bads:
            shards[i].buf[:] = 0
            shards[i] = shards[i].resliced(0)
        assert enc.reconstruct(shards, bads) == 0
        assert all(np.array_equal(a, b_) for a, b_ in zip(views(shards), origin))
    bads += list(range(t.N + t.M))
    assert enc.reconstruct([Slice(s.buf.copy(), s.len) for s in shards], bads) != 0
    for az in range(t.AZCount):
        locals_, n, m = t.LocalStripeInAZ(az)
        if locals_ is None:
            continue
        local = [shards[i] for i in locals_]
        lorigin = views(local)
        lb = []
        for b in range(n, n + m):
            lb.append(b)
            for i in lb:
                local[i].buf[:] = 0
                local[i] = local[i].resliced(0)
            assert enc.reconstruct(local, lb) == 0
            assert all(np.array_equal(a, b_) for a, b_ in zip(views(local), lorigin))
        if n > 0:
            lb.append(n - 1)
            assert enc.reconstruct(local, lb) != 0


def _digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:32]


@pytest.mark.parametrize("name", ["EC6P10L2", "EC16P20L2", "EC6P6", "EC12P4"])
def test_golden_mock_stripes_through_ec_oracle(name):
    t = cm.GetTactic(cm.ByName(name))
    enc = ECOracle.from_tactic(t, enable_verify=True)
    for row in GOLDEN["stripes"][name]:
        if row["size"] == 0:
            continue
        arr = [((row["bid"] + i + np.arange(row["size"])) & 0xFF).astype(np.uint8) for i in range(t.N)]
        shards = vector(arr + [np.zeros(row["size"], np.uint8)] * (t.M + t.L))
        assert enc.encode(shards) == 0
        assert [_digest(s.view()) for s in shards] == row["sha256"], (name, row["bid"])


def test_lrc_local_parity_is_the_local_engine_over_the_az():
    """lrcencoder.go:57-76: local parity = localEngine.Encode over [AZ data, AZ global parity]."""
    for mode in (cm.EC6P10L2, cm.EC16P20L2, cm.EC6P3L3, cm.EC4P4L2, cm.EC6P6L9, cm.EC6P8L10):
        t = cm.GetTactic(mode)
        rng = np.random.default_rng(mode)
        S = 1031
        arr = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(t.N)] + \
              [np.zeros(S, np.uint8) for _ in range(t.M + t.L)]
        shards = vector(arr)
        assert ECOracle.from_tactic(t).encode(shards) == 0
        glob = views(shards[:t.N + t.M])
        ref = [a.copy() for a in arr[:t.N]] + [np.zeros(S, np.uint8) for _ in range(t.M)]
        assert O.encode(t.N, t.M, ref) == 0
        assert all(np.array_equal(a, b) for a, b in zip(glob, ref))
        ln, lm = (t.N + t.M) // t.AZCount, t.L // t.AZCount
        for az in range(t.AZCount):
            idx, _, _ = t.LocalStripeInAZ(az)
            loc = [shards[i].view().copy() for i in idx[:ln]] + [np.zeros(S, np.uint8) for _ in range(lm)]
            assert O.encode(ln, lm, loc) == 0
            for j in range(lm):
                assert np.array_equal(loc[ln + j], shards[idx[ln + j]].view()), (mode, az, j)


# ------------------------------------------------------------------ quirks

def _lrc_codeword(t, S, seed):
    rng = np.random.default_rng(seed)
    arr = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(t.N)] + \
          [np.zeros(S, np.uint8) for _ in range(t.M + t.L)]
    sh = vector(arr)
    assert ECOracle.from_tactic(t).encode(sh) == 0
    return views(sh)


def test_missing_shard_outside_badidx_is_filled_not_rebuilt():
    """fillFullShards (encoder.go:199-210) gives a len-0 shard the shard size; Reconstruct only
    rebuilds badIdx, so a missing local parity outside badIdx keeps its cap bytes (or zeros when a
    fresh buffer had to be made) -- and Verify then reports the stripe bad."""
    t = cm.GetTactic(cm.EC6P10L2)
    enc = ECOracle.from_tactic(t)
    good = _lrc_codeword(t, 777, 1)
    L0 = t.N + t.M
    # cap 0: make([]byte, S) -> zeros
    sh = vector(good)
    sh[L0] = Slice()
    sh[2] = sh[2].resliced(0)
    assert enc.reconstruct(sh, [2]) == 0
    assert np.array_equal(sh[2].view(), good[2])
    assert sh[L0].len == 777 and not sh[L0].view().any()
    assert enc.verify(sh) == (False, 0)
    # cap >= S: the old bytes stay
    sh = vector(good)
    sh[L0].buf[:] = 0x77
    sh[L0] = sh[L0].resliced(0)
    assert enc.reconstruct(sh, [3]) == 0
    assert (sh[L0].view() == 0x77).all()
    # the same shard listed in badIdx is rebuilt by the AZ-local pass
    sh = vector(good)
    sh[L0] = Slice()
    assert enc.reconstruct(sh, [L0]) == 0
    assert np.array_equal(sh[L0].view(), good[L0])


def test_local_bad_idx_remap_and_global_first():
    """:161-171: local parity i of AZ idc is local index i - N - M - L/AZ*idc + (N+M)/AZ; the
    global pass runs first, so a bad local parity is rebuilt over the repaired global shards."""
    t = cm.GetTactic(cm.EC16P20L2)
    enc = ECOracle.from_tactic(t)
    good = _lrc_codeword(t, 4099, 2)
    for bad in ([0, 1, 16, 17, 36], [37], [5, 36, 37], [20, 35, 37]):
        sh = vector(good)
        for i in bad:
            sh[i].buf[:] = 0xA5  # broken bytes, full length (blobnode's bad shards)
        assert enc.reconstruct(sh, bad) == 0, bad
        assert all(np.array_equal(a, b) for a, b in zip(views(sh), good)), bad


def test_verify_order_and_errors():
    """:89-131: global Verify first (false -> return, locals never looked at), then every AZ."""
    t = cm.GetTactic(cm.EC6P10L2)
    enc = ECOracle.from_tactic(t)
    good = _lrc_codeword(t, 300, 3)
    sh = vector(good)
    assert enc.verify(sh) == (True, 0)
    sh[t.N + t.M + 1].buf[7] ^= 1
    assert enc.verify(sh) == (False, 0)
    sh = vector(good)
    sh[t.N + t.M] = Slice()  # a missing local parity: the global Verify passes, the local one errs
    assert enc.verify(sh) == (False, ERR_SHARD_SIZE)
    sh[t.N] = Slice()  # now the global Verify errs first
    assert enc.verify(sh) == (False, ERR_SHARD_SIZE)
    sh = vector(good)
    sh[0].buf[0] ^= 1
    sh[t.N + t.M] = Slice()  # global false returns before the local error
    assert enc.verify(sh) == (False, 0)
    ln = (t.N + t.M + t.L) // t.AZCount
    assert enc.verify(vector([good[i] for i in t.LocalStripeInAZ(1)[0]])) == (True, 0)
    assert len(t.LocalStripeInAZ(1)[0]) == ln


def test_reconstruct_errors_and_data_only():
    t = cm.GetTactic(cm.EC6P10L2)
    enc = ECOracle.from_tactic(t)
    good = _lrc_codeword(t, 64, 4)
    sh = vector(good)
    assert enc.reconstruct(sh, list(range(t.M + 1))) == ERR_TOO_FEW_SHARDS
    # ReconstructData leaves missing global parity and every local shard alone
    sh = vector(good)
    for i in (0, 7, t.N + t.M):
        sh[i] = Slice()
    assert enc.reconstruct_data(sh, [0, 7]) == 0
    assert np.array_equal(sh[0].view(), good[0])
    assert sh[7].len == 0  # filled by fillFullShards, emptied by initBadShards, not rebuilt (data only)
    assert sh[t.N + t.M].len == 0  # local shards are outside fillFullShards(shards[:N+M])
    sh = vector(good)
    sh[8] = Slice()
    assert enc.reconstruct_data(sh, [1]) == 0
    assert sh[8].len == 64 and not sh[8].view().any()  # a missing parity outside badIdx: zero-filled
    # a shard of another length
    sh = vector(good)
    sh[3] = Slice(np.zeros(63, np.uint8))
    assert enc.reconstruct(sh, [0]) == ERR_SHARD_SIZE


def test_rs_reconstruct_cap_reuse():
    """KRS/reedsolomon.go:1514-1518: a missing shard with enough cap is written in place."""
    k, m, S = 4, 2, 100
    rng = np.random.default_rng(5)
    arr = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.zeros(S, np.uint8)] * m
    sh = vector(arr)
    assert ECOracle(k, m).encode(sh) == 0
    good = views(sh)
    keep = sh[1].buf
    sh[1] = sh[1].resliced(0)
    sh[5] = Slice(np.zeros(S - 1, np.uint8), 0)  # cap short: a fresh buffer
    assert rs_reconstruct(k, m, sh) == 0
    assert sh[1].buf is keep and np.array_equal(sh[1].view(), good[1])
    assert sh[5].cap == S and np.array_equal(sh[5].view(), good[5])


def test_repair_status_matches_reconstruct_then_verify():
    t = cm.GetTactic(cm.EC16P20L2)
    enc = ECOracle.from_tactic(t)
    good = _lrc_codeword(t, 512, 6)
    r = random.Random(7)
    for _ in range(20):
        sh = vector(good)
        bad = sorted(r.sample(range(t.N + t.M + t.L), r.randint(1, 4)))
        j = r.randrange(t.N + t.M + t.L)
        if j not in bad and r.random() < 0.5:
            sh[j].buf[r.randrange(512)] ^= 0x10
        ref = [Slice(s.buf.copy(), s.len) for s in sh]
        st = enc.repair(sh, bad)
        err = enc.reconstruct(ref, bad)
        if err:
            assert st == err
            continue
        ok, err = enc.verify(ref)
        assert st == (err if err else (0 if ok else ERR_VERIFY))
        assert all(np.array_equal(a, b) for a, b in zip(views(sh), views(ref)))
