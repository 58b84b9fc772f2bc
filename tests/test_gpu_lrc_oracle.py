"""ec.Encoder (RS and LRC) single calls on the GPU against the ec oracle (oracle/ec_oracle.py), which
restates encoder.go / lrcencoder.go step by step over the RS oracle -- never against the GPU's own
results.  Inputs are deliberately inconsistent: corrupted data, global parity and local parity
shards (of either AZ), missing shards inside and outside badIdx, shards of the wrong length, local
stripes as inputs; sizes include C4's S = 699,051 and C5's S = 262,144.  Every case compares the
status and every shard's length and bytes.
"""
import random

import numpy as np
import pytest

from chubaofs_amd import _lib, codemode as cm
from oracle.ec_oracle import ECOracle, Slice

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

LRC_MODES = [cm.EC6P10L2, cm.EC16P20L2, cm.EC6P3L3, cm.EC4P4L2]
RS_MODES = [cm.EC6P6, cm.EC12P4, cm.EC15P12]
C4_S, C5_S = 699051, 262144


def new(mode, verify):
    from chubaofs_amd import ec
    return ec.NewEncoder(ec.Config(CodeMode=cm.GetTactic(mode), EnableVerify=verify), device=0)


def host(x):
    return x.cpu().numpy() if hasattr(x, "cpu") else np.asarray(x)


def to_mem(arrs, memory):
    if memory == "device":
        return [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]
    return [np.ascontiguousarray(a).copy() for a in arrs]


def to_oracle(arrs):
    """The Go view of what the Python mirror passes: a len-0 entry has no capacity (the mirror
    gives it a fresh zeroed buffer, as Go's make does)."""
    return [Slice() if a.size == 0 else Slice.of(a) for a in arrs]


def status_of(fn):
    try:
        r = fn()
    except _lib.CfsecError as e:
        return e.status, None
    return 0, r


def assert_same(got, want, ctx):
    got = [host(x) for x in got]
    assert len(got) == len(want), ctx
    for i, (g, w) in enumerate(zip(got, want)):
        assert g.size == w.len, (ctx, i, g.size, w.len)
        assert np.array_equal(g, w.view()), (ctx, i)


def codeword(t, S, seed):
    rng = np.random.default_rng(seed)
    arr = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(t.N)] + \
          [np.zeros(S, np.uint8) for _ in range(t.M + t.L)]
    sh = to_oracle(arr)
    assert ECOracle.from_tactic(t).encode(sh) == 0
    return [s.view().copy() for s in sh]


def damage(t, good, r, kinds):
    """A copy of `good` with the listed damages: ('flip', i) a byte of shard i, ('drop', i) a
    missing shard (len 0), ('len', i) shard i one byte longer."""
    arrs = [g.copy() for g in good]
    for kind, i in kinds:
        if kind == "flip" and arrs[i].size:
            arrs[i][r.randrange(arrs[i].size)] ^= 1 + r.randrange(255)
        elif kind == "drop":
            arrs[i] = arrs[i][:0]
        elif kind == "len":
            arrs[i] = np.concatenate([arrs[i], np.zeros(1, np.uint8)])
    return arrs


def random_damage(t, r, total, n_flip, n_drop):
    idx = list(range(total))
    r.shuffle(idx)
    return [("flip", i) for i in idx[:n_flip]] + [("drop", i) for i in idx[n_flip:n_flip + n_drop]]


def run_case(mode, op, arrs, bad, memory, verify_on=True):
    t = cm.GetTactic(mode)
    enc = new(mode, verify_on)
    orc = ECOracle.from_tactic(t, enable_verify=verify_on)
    work = to_mem(arrs, memory)
    want = to_oracle(arrs)
    if op == "encode":
        st, _ = status_of(lambda: enc.Encode(work))
        exp = orc.encode(want)
    elif op == "verify":
        st, ok = status_of(lambda: enc.Verify(work))
        ok_w, exp = orc.verify(want)
        if st == 0 and exp == 0:
            assert ok == ok_w, (cm.Name(mode), op, bad)
    elif op == "reconstruct":
        st, _ = status_of(lambda: enc.Reconstruct(work, bad))
        exp = orc.reconstruct(want, bad)
    else:
        st, _ = status_of(lambda: enc.ReconstructData(work, bad))
        exp = orc.reconstruct_data(want, bad)
    ctx = (cm.Name(mode), op, memory, bad, [a.size for a in arrs][:4])
    assert st == exp, (ctx, st, exp)
    assert_same(work, want, ctx)


@pytest.mark.parametrize("memory", ["host", "device"])
@pytest.mark.parametrize("mode", LRC_MODES + RS_MODES)
def test_random_inconsistent_ops(mode, memory):
    t = cm.GetTactic(mode)
    total = t.N + t.M + t.L
    r = random.Random(mode * 31 + (memory == "device"))
    for case in range(24):
        S = r.choice([1, 23, 4096, 4097, 65537])
        good = codeword(t, S, case)
        op = ["encode", "verify", "reconstruct", "reconstruct_data"][case % 4]
        kinds = random_damage(t, r, total, r.randint(0, 2), r.randint(0, 2))
        if op == "encode":
            kinds = [k for k in kinds if k[1] >= t.N or k[0] == "drop"]  # data intact or missing
        bad = sorted(r.sample(range(total), r.randint(0, max(1, t.M // 2)))) if "recon" in op else []
        run_case(mode, op, damage(t, good, r, kinds), bad, memory)


@pytest.mark.parametrize("memory", ["host", "device"])
@pytest.mark.parametrize("mode", [cm.EC6P10L2, cm.EC16P20L2])
def test_lrc_targeted(mode, memory):
    """The lrcencoder.go paths one by one."""
    t = cm.GetTactic(mode)
    N, M, L = t.N, t.M, t.L
    L0, L1 = N + M, N + M + L - 1
    r = random.Random(mode)
    S = 4097
    good = codeword(t, S, 11)
    cases = [
        # Verify: global first, early return (:101-107), then each AZ (:109-130)
        ("verify", [], []), ("verify", [("flip", L0)], []), ("verify", [("flip", L1)], []),
        ("verify", [("flip", N + M - 1)], []), ("verify", [("flip", 0), ("drop", L0)], []),
        ("verify", [("drop", L1)], []), ("verify", [("drop", N)], []), ("verify", [("len", L0)], []),
        # Reconstruct: global then the local remap (:161-171)
        ("reconstruct", [], [0, L0]), ("reconstruct", [], [L0, L1]), ("reconstruct", [], [N, L1]),
        ("reconstruct", [("drop", L0)], [1]),          # missing local parity outside badIdx: filled
        ("reconstruct", [("drop", 2)], [2, L1]),
        ("reconstruct", [("flip", 3)], [0, L0]),       # a corrupted input propagates
        ("reconstruct", [("flip", N)], [L1]),          # a local rebuilt from a corrupted global parity
        ("reconstruct", [], list(range(M + 1))),       # ErrTooFewShards
        ("reconstruct", [("len", L0)], [0]),           # a local shard of another length
        # ReconstructData (:188-201)
        ("reconstruct_data", [("drop", L0), ("drop", N + 1)], [0]), ("reconstruct_data", [], [0, N, L0]),
        # Encode: fill (:41), global, locals; a local of the wrong length (global still written)
        ("encode", [("drop", L0), ("drop", N)], []), ("encode", [("drop", 0)], []),
        ("encode", [("len", L1)], []), ("encode", [("len", N)], []),
    ]
    for op, kinds, bad in cases:
        run_case(mode, op, damage(t, good, r, kinds), bad, memory)
        run_case(mode, op, damage(t, good, r, kinds), bad, memory, verify_on=False)


@pytest.mark.parametrize("mode", LRC_MODES)
def test_local_stripe_inputs(mode):
    """A local stripe as the shard vector (lrcencoder.go:93-99, 147-152): local Verify and Reconstruct
    of every position, with corrupted members."""
    t = cm.GetTactic(mode)
    good = codeword(t, 1000 + mode, mode)
    r = random.Random(mode)
    for az in range(t.AZCount):
        idx, _, _ = t.LocalStripeInAZ(az)
        local = [good[i] for i in idx]
        n = len(local)
        for pos in range(n):
            run_case(mode, "reconstruct", damage(t, local, r, [("flip", pos)]), [pos], "host")
            run_case(mode, "verify", damage(t, local, r, [("flip", pos)]), [], "host")
        run_case(mode, "reconstruct", damage(t, local, r, [("flip", 0)]), [n - 1], "device")
        run_case(mode, "reconstruct", local, list(range(n)), "device")


@pytest.mark.parametrize("memory", ["host", "device"])
def test_c4_c5_sizes(memory):
    """C4 (EC6P10L2, S = 699,051: AZ-local repair) and C5 (EC16P20L2, S = 262,144: {0,1,16,17})."""
    r = random.Random(45)
    t4 = cm.GetTactic(cm.EC6P10L2)
    good = codeword(t4, C4_S, 4)
    L0 = t4.N + t4.M
    run_case(cm.EC6P10L2, "encode", damage(t4, good, r, [("drop", L0)]), [], memory)
    run_case(cm.EC6P10L2, "reconstruct", damage(t4, good, r, [("flip", L0 + 1)]), [L0], memory)
    idx, _, _ = t4.LocalStripeInAZ(0)
    run_case(cm.EC6P10L2, "reconstruct", damage(t4, [good[i] for i in idx], r, [("flip", 2)]), [2], memory)
    t5 = cm.GetTactic(cm.EC16P20L2)
    good = codeword(t5, C5_S, 5)
    for kinds in ([], [("flip", 36)], [("flip", 37)], [("flip", 35)], [("flip", 5)]):
        run_case(cm.EC16P20L2, "reconstruct", damage(t5, good, r, kinds), [0, 1, 16, 17], memory)
        run_case(cm.EC16P20L2, "verify", damage(t5, good, r, kinds), [], memory)


@pytest.mark.parametrize("memory", ["host", "device"])
@pytest.mark.parametrize("mode", [cm.EC6P6L9, cm.EC6P8L10])
def test_local_pass_failure_runs_every_az(mode, memory):
    """lrcencoder.go:173-184 hands every AZ's local Reconstruct to task.Run, which runs them all and
    returns the first error: when AZ 0's local pass fails (another local parity of AZ 0 has the wrong
    length: ErrShardSize) AZ 1's bad local parity is still rebuilt.  Single call and the tasklet
    batch, both against the ec oracle (status, lengths and bytes)."""
    t = cm.GetTactic(mode)
    N, M, L, AZ = t.N, t.M, t.L, t.AZCount
    lpa = L // AZ
    az0, az1 = N + M, N + M + lpa  # first local parity of AZ 0 and of AZ 1
    r = random.Random(mode)
    good = codeword(t, 2049, 77)
    cases = [
        ([("len", az0 + 1), ("flip", az1)], [az0, az1]),   # AZ 0 fails, AZ 1 rebuilt
        ([("len", az1 + 1), ("flip", az0)], [az0, az1]),   # AZ 1 fails, AZ 0 rebuilt
        ([("len", az0 + 1), ("len", az1 + 1)], [az0, az1]),  # both fail: AZ 0's error
        ([("flip", az1)], [az0, az1]),                      # both rebuilt
    ]
    for kinds, bad in cases:
        run_case(mode, "reconstruct", damage(t, good, r, kinds), bad, memory)
    # the tasklet form: the same bids in one cfsec_ec_reconstruct_batch (Reconstruct + Verify per bid)
    enc = new(mode, False)
    bids = [damage(t, good, random.Random(i), kinds) for i, (kinds, _) in enumerate(cases)]
    want = [to_oracle(b) for b in bids]
    orc = ECOracle.from_tactic(t)
    exp = [orc.repair(w, bad) for w, (_, bad) in zip(want, cases)]
    work = [to_mem(b, memory) for b in bids]
    st = enc.ReconstructBatch(work, [bad for _, bad in cases], verify=True)
    assert st == exp, (cm.Name(mode), st, exp)
    for b, (wk, w) in enumerate(zip(work, want)):
        if exp[b] in (0, _lib.ErrVerify.status):
            assert_same(wk, w, (cm.Name(mode), "batch", b))


@pytest.mark.parametrize("S", [2048, 2048 * 3 + 16, 262144 + 2048 + 48])
def test_ec16p20l2_encode_bitsliced_column_runs(S):
    """EC16P20L2's fused encode of 16-byte-aligned rows takes the bit-sliced network for the whole
    2 KiB column runs and the dyadic kernel for the rest of each row (gf_bs16.hip; S = 2048: no
    rest, S = 6160: 16 bytes of rest): every shard against the ec oracle, as single calls on
    separate shard tensors and as a batch over one [bids, 38, S] buffer with stale parity."""
    t = cm.GetTactic(cm.EC16P20L2)
    n = t.N + t.M + t.L
    good = [codeword(t, S, 70 + b) for b in range(3)]
    for b in range(2):
        arrs = [g.copy() for g in good[b]]
        for a in arrs[t.N:]:
            a[:] = 0xA5
        run_case(cm.EC16P20L2, "encode", arrs, [], "device", verify_on=False)
    buf = torch.empty((3, n, S), dtype=torch.uint8, device="cuda")
    for b in range(3):
        for i in range(n):
            buf[b, i] = torch.from_numpy(good[b][i] if i < t.N else np.full(S, 0x5A, np.uint8))
    assert buf.data_ptr() % 16 == 0 and (S % 16 == 0)
    st = new(cm.EC16P20L2, False).EncodeBatch([[buf[b, i] for i in range(n)] for b in range(3)])
    assert st == [0, 0, 0]
    got = buf.cpu().numpy()
    for b in range(3):
        for i in range(n):
            assert np.array_equal(got[b, i], good[b][i]), (S, b, i)
