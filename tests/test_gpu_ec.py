"""ec.Encoder / lrcEncoder on the GPU, mirroring blobstore/common/ec/encoder_test.go and the
blobnode repair loop (work_shard_recover.go:708-771), in host and device memory.

Round trips are the reference's own invariants (reflect.DeepEqual after Reconstruct, Verify
true/false); on top, every parity byte is compared with the oracle (global parity =
oracle encode; local parity = oracle encode of the AZ's local stripe with the local engine).
"""
import io
import random

import numpy as np
import pytest

from chubaofs_amd import _lib, codemode as cm
from oracle import oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

SRC = np.frombuffer(b"Hello world", np.uint8)


def ec_mod():
    from chubaofs_amd import ec
    return ec


def new(mode, verify=True, conc=0):
    ec = ec_mod()
    return ec.NewEncoder(ec.Config(CodeMode=cm.GetTactic(mode), EnableVerify=verify, Concurrency=conc))


def to_dev(shards):
    return [torch.from_numpy(np.ascontiguousarray(s)).cuda() for s in shards]


def host(shards):
    torch.cuda.synchronize()
    return [s.cpu().numpy() if hasattr(s, "cpu") else s for s in shards]


def copy_shards(shards):
    return [s.clone() if hasattr(s, "clone") else s.copy() for s in shards]


def expected_parity(mode, shards_host):
    """Global parity + every AZ's local parity from the oracle (lrcencoder.go:35-82)."""
    t = cm.GetTactic(mode)
    full = [s.copy() for s in shards_host]
    assert O.encode(t.N, t.M, full[:t.N + t.M]) == 0
    if t.L:
        ln, lm = (t.N + t.M) // t.AZCount, t.L // t.AZCount
        for az in range(t.AZCount):
            idx, _, _ = t.LocalStripeInAZ(az)
            local = [full[i] for i in idx]
            assert O.encode(ln, lm, local) == 0
    return full


@pytest.mark.parametrize("memory", ["host", "device"])
def test_encoder_ec15p12(memory):
    """encoder_test.go:53-106 (TestEncoder)."""
    enc = new(cm.EC15P12)
    t = enc.CodeMode
    shards = enc.Split(SRC.copy())
    if memory == "device":
        shards = to_dev(shards)
    enc.Encode(shards)
    want = expected_parity(cm.EC15P12, host(shards))
    assert all(np.array_equal(a, b) for a, b in zip(host(shards), want))
    buf = io.BytesIO()
    enc.Join(buf, host(shards), len(SRC))
    assert buf.getvalue() == SRC.tobytes()
    data = enc.GetDataShards(shards)
    data[0][:] = 222
    enc.ReconstructData(shards, [0])
    buf = io.BytesIO()
    enc.Join(buf, host(shards), len(SRC))
    assert buf.getvalue() == SRC.tobytes()
    parity = enc.GetParityShards(shards)
    parity[1][:] = 11
    enc.Reconstruct(shards, [t.N + 1])
    assert enc.Verify(shards)
    assert all(np.array_equal(a, b) for a, b in zip(host(shards), want))
    assert enc.GetLocalShards(shards) == []
    assert len(enc.GetShardsInIdc(list(shards), 0)) == (t.N + t.M) // 3


@pytest.mark.parametrize("memory", ["host", "device"])
def test_lrc_encoder_ec6p10l2(memory):
    """encoder_test.go:108-247 (TestLrcEncoder)."""
    enc = new(cm.EC6P10L2)
    t = enc.CodeMode
    with pytest.raises(_lib.ErrShortData):
        enc.Split(np.zeros(0, np.uint8))
    shards = enc.Split(SRC.copy())
    big = np.zeros(1 << 10, np.uint8)
    big[:len(SRC)] = SRC
    assert len(enc.Split(big, len(SRC))) == 18
    if memory == "device":
        shards = to_dev(shards)
    with pytest.raises(_lib.ErrInvalidShards):
        enc.Encode(shards[:-1])
    enc.Encode(shards)
    want = expected_parity(cm.EC6P10L2, host(shards))
    assert all(np.array_equal(a, b) for a, b in zip(host(shards), want)), "LRC parity differs from oracle"
    buf = io.BytesIO()
    enc.Join(buf, host(shards), len(SRC))
    assert buf.getvalue() == SRC.tobytes()

    enc.GetDataShards(shards)[0][:] = 222
    assert not enc.Verify(shards)
    enc.ReconstructData(shards, [0])
    buf = io.BytesIO()
    enc.Join(buf, host(shards), len(SRC))
    assert buf.getvalue() == SRC.tobytes()

    # local reconstruct of every position of AZ0's local stripe
    local = enc.GetShardsInIdc(shards, 0)
    for idx in range(len(local)):
        local[idx][:] = 11
        assert not enc.Verify(shards)
        enc.Reconstruct(local, [idx])
        assert enc.Verify(shards)

    bad = []
    shards[t.N + t.M + 1][:] = 222
    bad.append(t.N + t.M + 1)
    assert not enc.Verify(shards)
    data, parity = enc.GetDataShards(shards), enc.GetParityShards(shards)
    for i in range(t.M):
        if i % 2 == 0:
            bad.append(i)
            if i < len(data):
                data[i][:] = 222
        else:
            bad.append(t.N + i)
            parity[i][:] = 222
    assert not enc.Verify(shards)
    enc.Reconstruct(shards, bad)
    assert enc.Verify(shards)
    assert all(np.array_equal(a, b) for a, b in zip(host(shards), want))
    assert len(enc.GetLocalShards(shards)) == t.L
    assert len(enc.GetShardsInIdc(shards, 0)) == (t.N + t.M + t.L) // t.AZCount

    # zero-length shard: Verify errors (checkShards), Reconstruct refills it
    shards[bad[0]] = shards[bad[0]][:0]
    with pytest.raises(_lib.ErrShardSize):
        enc.Verify(shards)
    enc.Reconstruct(shards, bad)
    assert enc.Verify(shards)


@pytest.mark.parametrize("mode", cm.GetAllCodeModes())
@pytest.mark.parametrize("memory", ["host", "device"])
def test_lrc_reconstruct_all_modes(mode, memory):
    """encoder_test.go:249-307 (TestLrcReconstruct) with random 64-128 KiB data."""
    t = cm.GetTactic(mode)
    enc = new(mode)
    rng = np.random.default_rng(mode)
    data = rng.integers(0, 256, (1 << 16) + int(rng.integers(0, 1 << 16)), dtype=np.uint8)
    shards = enc.Split(data)
    if memory == "device":
        shards = to_dev(shards)
    enc.Encode(shards)
    origin = host(copy_shards(shards))
    want = expected_parity(mode, origin)
    assert all(np.array_equal(a, b) for a, b in zip(origin, want)), "parity differs from oracle"
    bads = []
    for bad in range(t.N + t.M, t.N + t.M + t.L):
        bads.append(bad)
        for i in bads:
            shards[i][:] = 0
            shards[i] = shards[i][:0]
        enc.Reconstruct(shards, bads)
        assert all(np.array_equal(a, b) for a, b in zip(host(shards), origin))
    for bad in range(t.N + t.M):
        bads.append(bad)
    # every global shard bad: checkShards sees no data (ErrShardNoData); the Go test only
    # requires an error here
    with pytest.raises(_lib.CfsecError):
        enc.Reconstruct(copy_shards(shards), bads)
    for az in range(t.AZCount):
        locals_, n, m = t.LocalStripeInAZ(az)
        if locals_ is None:
            continue
        local = [shards[i] for i in locals_]
        lorigin = host(copy_shards(local))
        lbad = []
        for b in range(n, n + m):
            lbad.append(b)
            for i in lbad:
                local[i][:] = 0
                local[i] = local[i][:0]
            enc.Reconstruct(local, lbad)
            assert all(np.array_equal(a, b_) for a, b_ in zip(host(local), lorigin))
        if n > 0:
            lbad.append(n - 1)
            with pytest.raises(_lib.ErrTooFewShards):
                enc.Reconstruct(local, lbad)


def gen_mock_bytes(letter, size):
    """blobnode/worker_for_test.go:62-69"""
    return np.array([(letter + i) & 0xFF for i in range(size)], np.uint8)


@pytest.mark.parametrize("mode", [cm.EC6P6, cm.EC12P4, cm.EC6P10L2, cm.EC16P20L2, cm.EC15P12, cm.EC4P4L2])
def test_blobnode_repair_loop_mock_bids(mode):
    """work_shard_recover.go:708-771 over worker_for_test.go's bids {1024,2048,0,512,23,65,12}:
    Reconstruct(blobShards, recoverIdx) then Verify, per bid; zero-size bids are skipped there."""
    t = cm.GetTactic(mode)
    enc = new(mode, verify=False)
    total = t.N + t.M + t.L
    r = random.Random(mode)
    for size in (1024, 2048, 512, 23, 65, 12):
        shards = [gen_mock_bytes(ord("A") + i, size) for i in range(t.N)] + \
                 [np.zeros(size, np.uint8) for _ in range(total - t.N)]
        dev = to_dev(shards)
        enc.Encode(dev)
        good = host(dev)
        assert all(np.array_equal(a, b) for a, b in zip(good, expected_parity(mode, good)))
        nbad = r.randint(1, t.M)
        recover = sorted(r.sample(range(total), nbad))
        for i in recover:
            dev[i][:] = 0  # the broken shard's buffer, still full length
        enc.Reconstruct(dev, recover)
        assert enc.Verify(dev)
        assert all(np.array_equal(a, b) for a, b in zip(host(dev), good)), (size, recover)


def test_concurrent_encoders_threads():
    """One encoder shared by many goroutines (encoder.go:90): concurrent calls from threads."""
    import concurrent.futures as cf
    enc = new(cm.EC12P4, verify=True, conc=4)
    rng = np.random.default_rng(9)

    def job(seed):
        data = np.random.default_rng(seed).integers(0, 256, 300000 + seed, dtype=np.uint8)
        shards = enc.Split(data)
        enc.Encode(shards)
        want = expected_parity(cm.EC12P4, shards)
        assert all(np.array_equal(a, b) for a, b in zip(shards, want))
        orig = [s.copy() for s in shards]
        bad = sorted(np.random.default_rng(seed).choice(16, 4, replace=False).tolist())
        for i in bad:
            shards[i] = shards[i][:0]
        enc.Reconstruct(shards, bad)
        return all(np.array_equal(a, b) for a, b in zip(shards, orig))

    with cf.ThreadPoolExecutor(8) as ex:
        assert all(ex.map(job, range(24)))
    del rng


@pytest.mark.parametrize("mode", [cm.EC6P6, cm.EC12P4, cm.EC6P10L2, cm.EC16P20L2])
@pytest.mark.parametrize("memory", ["host", "device"])
def test_segment_reconstruct_data(mode, memory):
    """access/stream_get.go:420-431: a ranged Get rebuilds only the requested byte range of the
    data shards -- ReconstructData over sub-slices shards[i][off:off+size] of the full shards,
    with the bad shards' segments rebuilt in place inside the original buffers."""
    t = cm.GetTactic(mode)
    enc = new(mode, verify=False)
    rng = np.random.default_rng(mode * 7 + (memory == "device"))
    data = rng.integers(0, 256, 200003, dtype=np.uint8)
    shards = enc.Split(data)
    if memory == "device":
        shards = to_dev(shards)
    enc.Encode(shards)
    origin = host(copy_shards(shards))
    S = len(origin[0])
    for off, size in [(0, 1), (17, 4096), (S // 3, 1000), (S - 5, 5), (4095, 8193)]:
        size = min(size, S - off)
        bad = sorted(rng.choice(t.N + t.M, t.M, replace=False).tolist())
        work = copy_shards(shards)
        for i in bad:
            work[i][off:off + size] = 0  # the bad shards' bytes in the range are unknown
        segments = [s[off:off + size] for s in work]
        enc.ReconstructData(segments, bad)
        got = host(work)
        for i in range(t.N):  # every data segment restored, inside the original buffer
            assert np.array_equal(got[i][off:off + size], origin[i][off:off + size]), (off, size, i, bad)
        for i in range(t.N + t.M + t.L):  # nothing outside the range was touched
            assert np.array_equal(got[i][:off], origin[i][:off] if i not in bad else got[i][:off])
            assert np.array_equal(got[i][off + size:], origin[i][off + size:]), (off, size, i)


@pytest.mark.gpu
def test_repair_rows_match_reconstruct_and_errors():
    """cfsec_ec_repair_rows: rows over the first N present global shards reproduce every erased
    shard (data, global and local parity) through cfsec_ec_matvec_batch; out-of-range and
    too-many-lost sets are refused with the reference's errors."""
    import torch
    from chubaofs_amd import _lib, codemode as cm, ec
    t = cm.GetTactic(cm.EC6P10L2)
    enc = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=False), device=0)
    total, S = t.N + t.M + t.L, 4096 + 5
    rng = np.random.default_rng(9)
    sh = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(t.N)] + [np.zeros(S, np.uint8) for _ in range(t.M + t.L)]
    enc.Encode(sh)
    bad = [0, 3, 7, 16]
    ins, rows = enc.repair_rows(bad, bad)
    assert ins == [i for i in range(t.N + t.M) if i not in bad][:t.N]
    dev = torch.from_numpy(np.stack(sh)).cuda()
    out = torch.zeros((len(bad), S), dtype=torch.uint8, device="cuda")
    ptrs = [dev[i].data_ptr() for i in ins] + [out[q].data_ptr() for q in range(len(bad))]
    enc.matvec_batch(rows, ptrs, S, 1)
    torch.cuda.synchronize()
    for q, e in enumerate(bad):
        assert np.array_equal(out[q].cpu().numpy(), sh[e]), e
    with pytest.raises(_lib.CfsecError):
        enc.repair_rows([total], [0])
    with pytest.raises(_lib.CfsecError):
        enc.repair_rows(list(range(t.M + 1)), [0])  # 11 global shards lost, 5 left < N = 6
