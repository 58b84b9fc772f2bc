"""GPU parity: the gfx950 engine (through the C ABI) against the CPU oracle.

Bit-exact equality is the bar for every byte (integer GF(2^8) work).  The oracle
(oracle/gf_oracle.c) restates klauspost/reedsolomon v1.11.7 and is pinned by the
reference's literal field tables (tests/test_oracle.py).
"""
import itertools
import random

import numpy as np
import pytest

from oracle import oracle as O

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

MODES_KM = [(6, 6), (12, 4), (6, 10), (8, 1), (16, 20), (18, 1), (15, 12), (3, 3), (16, 4), (10, 4),
            (4, 4), (6, 3), (12, 9), (1, 1), (2, 5)]
SIZES = [1, 15, 16, 17, 100, 4095, 4096, 4097, 65539, 174763]


def rng(seed):
    return np.random.default_rng(seed)


def rand_shards(k, m, size, seed):
    r = rng(seed)
    return [r.integers(0, 256, size, dtype=np.uint8) for _ in range(k)] + [np.zeros(size, np.uint8) for _ in range(m)]


def to_dev(arrs):
    return [None if a is None else torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


def to_host(ts):
    torch.cuda.synchronize()
    return [None if t is None else t.cpu().numpy() for t in ts]


def oracle_encoded(k, m, size, seed):
    sh = rand_shards(k, m, size, seed)
    assert O.encode(k, m, sh) == 0
    return sh


@pytest.fixture(scope="module")
def rs():
    from chubaofs_amd import reedsolomon
    return reedsolomon


_ENGINES = {}


def engine(rs, k, m):
    """One engine per (k, m), shared like the access/blobnode encoder pools."""
    if (k, m) not in _ENGINES:
        _ENGINES[(k, m)] = rs.New(k, m)
    return _ENGINES[(k, m)]


@pytest.mark.parametrize("k,m", MODES_KM)
@pytest.mark.parametrize("size", SIZES)
def test_encode_device_matches_oracle(rs, k, m, size):
    want = oracle_encoded(k, m, size, seed=k * 1000 + m * 10 + size)
    sh = [s.copy() for s in want]
    for p in sh[k:]:
        p[:] = 0xA5  # stale parity must be overwritten
    d = to_dev(sh)
    rs.New(k, m).Encode(d)
    got = to_host(d)
    for i in range(k + m):
        assert np.array_equal(got[i], want[i]), f"shard {i} differs (k={k} m={m} size={size})"


@pytest.mark.parametrize("k,m", [(12, 4), (6, 6), (16, 20)])
@pytest.mark.parametrize("size", [1, 17, 4097, 100003])
def test_encode_host_memory(rs, k, m, size):
    want = oracle_encoded(k, m, size, seed=7 + size)
    sh = [s.copy() for s in want]
    for p in sh[k:]:
        p[:] = 0
    rs.New(k, m).Encode(sh)
    for i in range(k + m):
        assert np.array_equal(sh[i], want[i])


@pytest.mark.parametrize("S", [5, 4097, 349526, 174763])
def test_encode_misaligned_contiguous_stripe(rs, S):
    """Shards carved at stride S from one buffer (ec.Buffer layout, buf.go:83-84): rows start
    at arbitrary byte offsets, like blobnode/access buffers."""
    k, m = 12, 4
    r = rng(S)
    buf = r.integers(0, 256, (k + m) * S + 3, dtype=np.uint8)
    dbuf = torch.from_numpy(buf).cuda()
    base = 3  # also misalign the stripe start
    shards = [dbuf[base + i * S: base + (i + 1) * S] for i in range(k + m)]
    rs.New(k, m).Encode(shards)
    want = [buf[base + i * S: base + (i + 1) * S].copy() for i in range(k + m)]
    assert O.encode(k, m, want) == 0
    got = dbuf.cpu().numpy()
    for i in range(k + m):
        assert np.array_equal(got[base + i * S: base + (i + 1) * S], want[i])
    assert np.array_equal(got[:base], buf[:base]) and np.array_equal(got[base + (k + m) * S:], buf[base + (k + m) * S:])


@pytest.mark.parametrize("k,m,size", [(12, 4, 4097), (6, 6, 1), (16, 20, 333), (40, 3, 1000)])
def test_verify_detects_every_single_byte_flip_position_class(rs, k, m, size):
    sh = oracle_encoded(k, m, size, seed=size)
    enc = rs.New(k, m)
    d = to_dev(sh)
    assert enc.Verify(d)
    r = random.Random(size)
    for trial in range(12):
        idx = r.randrange(k + m)
        pos = r.randrange(size)
        bad = [s.copy() for s in sh]
        bad[idx][pos] ^= 1 << r.randrange(8)
        assert not enc.Verify(to_dev(bad)), (idx, pos)
        assert O.verify(k, m, bad) == (0, False)


def test_encode_many_inputs_chunked(rs):
    """k > 32 takes the input-chunked accumulate path of the launcher."""
    k, m, size = 40, 3, 5000
    want = oracle_encoded(k, m, size, seed=40)
    d = to_dev([s.copy() for s in want])
    rs.New(k, m).Encode(d)
    got = to_host(d)
    for i in range(k, k + m):
        assert np.array_equal(got[i], want[i])


FIXED_MAX_M = {3: 6, 4: 6, 6: 12, 7: 6, 8: 8, 10: 6, 12: 12, 15: 12, 16: 24, 18: 4}  # gf_launch.hpp fixed_max_m


@pytest.mark.parametrize("k,m", [(k, m) for k, top in FIXED_MAX_M.items() for m in range(1, top + 2)])
def test_every_fixed_kernel_output_count(rs, k, m):
    """Every output count of the fixed-K kernels (plain and dyadic-block, store and verify), plus the
    first count past them (runtime-k kernel): encode, verify with and without a flipped parity
    byte, the worst-case data erasure (coset-aligned, dyadic for k = 6, 12, 16) and a random
    erasure set of size m (a general matrix) -- all against the oracle."""
    size = 8209  # two 4 KiB tiles + a ragged tail
    want = oracle_encoded(k, m, size, seed=k * 64 + m)
    enc = rs.New(k, m)
    d = to_dev([s if i < k else np.full(size, 0x5A, np.uint8) for i, s in enumerate(want)])
    enc.Encode(d)
    got = to_host(d)
    for i in range(k, k + m):
        assert np.array_equal(got[i], want[i]), i
    assert enc.Verify(d)
    d[k + m - 1][size - 1] ^= 0x10
    assert not enc.Verify(d)
    r = random.Random(k * 100 + m)
    for erased in (set(range(min(m, k))), set(r.sample(range(k + m), m))):
        _check_recon(rs, k, m, size, erased, False, seed=m)


def _check_recon(rs, k, m, size, erased, data_only, seed, consistent=True):
    if consistent:
        full = oracle_encoded(k, m, size, seed)
    else:  # arbitrary bytes: the fused single pass must still match the two-pass reference
        r = rng(seed)
        full = [r.integers(0, 256, size, dtype=np.uint8) for _ in range(k + m)]
    present = [i not in erased for i in range(k + m)]
    want = [s.copy() for s in full]
    for i in erased:
        want[i][:] = 0
    err, filled = O.reconstruct(k, m, want, present, data_only)
    dev = to_dev([s if p else s[:0] for s, p in zip(full, present)])
    enc = engine(rs, k, m)
    if err:
        from chubaofs_amd._lib import ErrTooFewShards
        assert err == ErrTooFewShards.status
        with pytest.raises(ErrTooFewShards):
            (enc.ReconstructData if data_only else enc.Reconstruct)(dev)
        return
    (enc.ReconstructData if data_only else enc.Reconstruct)(dev)
    got = to_host(dev)
    for i in range(k + m):
        if present[i] or filled[i]:
            assert got[i].size == size and np.array_equal(got[i], want[i]), (i, erased)
        else:
            assert got[i].size == 0, (i, erased)


def test_reconstruct_every_erasure_pattern_ec12p4(rs):
    k, m, size = 12, 4, 67
    n = 0
    for e in range(1, 5):
        for erased in itertools.combinations(range(16), e):
            _check_recon(rs, k, m, size, set(erased), False, seed=n)
            n += 1
    assert n == 2516


@pytest.mark.parametrize("k,m", MODES_KM)
@pytest.mark.parametrize("data_only", [False, True])
def test_reconstruct_random_patterns(rs, k, m, data_only):
    r = random.Random(k * 31 + m)
    for trial in range(6):
        e = r.randint(1, m + (1 if trial == 5 else 0))  # last trial may exceed m -> ErrTooFewShards
        erased = set(r.sample(range(k + m), min(e, k + m)))
        size = r.choice([1, 16, 33, 4100, 9999])
        _check_recon(rs, k, m, size, erased, data_only, seed=trial)


@pytest.mark.parametrize("k,m", [(12, 4), (6, 10), (16, 20)])
def test_reconstruct_inconsistent_inputs_bit_exact(rs, k, m):
    """Survivors that are NOT a codeword: reference pass 2 re-encodes parity from the rebuilt data;
    the fused pass uses parity x inv(sub).  Same linear map -> identical bytes."""
    r = random.Random(k)
    for trial in range(8):
        erased = set(r.sample(range(k + m), r.randint(1, m)))
        _check_recon(rs, k, m, 513, erased, False, seed=100 + trial, consistent=False)


def test_reconstruct_too_few(rs):
    from chubaofs_amd._lib import ErrTooFewShards
    k, m = 12, 4
    full = oracle_encoded(k, m, 100, 1)
    d = to_dev(full)
    for i in range(5):
        d[i] = d[i][:0]
    with pytest.raises(ErrTooFewShards):
        rs.New(k, m).Reconstruct(d)


def _stripe_batch(k, m, S, nstripes, seed):
    total = k + m
    pitch = (S + 255) // 256 * 256
    r = rng(seed)
    host = np.zeros((nstripes, total, pitch), np.uint8)
    host[:, :k, :S] = r.integers(0, 256, (nstripes, k, S), dtype=np.uint8)
    dev = torch.from_numpy(host).cuda()
    base = dev.data_ptr()
    ptrs = [base + (s * total + i) * pitch for s in range(nstripes) for i in range(total)]
    return host, dev, ptrs, pitch


@pytest.mark.parametrize("k,m,S,nstripes", [(12, 4, 100000, 5), (6, 6, 174763, 3), (16, 20, 4097, 9),
                                             (12, 4, 7, 40)])
def test_batch_encode_verify_reconstruct(rs, k, m, S, nstripes):
    host, dev, ptrs, pitch = _stripe_batch(k, m, S, nstripes, seed=S)
    enc = rs.New(k, m)
    enc.encode_batch(ptrs, S, nstripes)
    got = dev.cpu().numpy()
    for s in range(nstripes):
        want = [host[s, i, :S].copy() for i in range(k + m)]
        assert O.encode(k, m, want) == 0
        for i in range(k + m):
            assert np.array_equal(got[s, i, :S], want[i]), (s, i)
    flags = torch.zeros(nstripes, dtype=torch.int32, device="cuda")
    enc.verify_batch(ptrs, S, nstripes, flags.data_ptr())
    assert flags.cpu().numpy().tolist() == [0] * nstripes
    # corrupt stripe 1's last parity byte and stripe 0's first data byte
    dev[1, k + m - 1, S - 1] ^= 0x40
    dev[0, 0, 0] ^= 1
    flags.zero_()
    enc.verify_batch(ptrs, S, nstripes, flags.data_ptr())
    fl = flags.cpu().numpy().tolist()
    assert fl[0] == 1 and fl[1] == 1 and fl[2:] == [0] * (nstripes - 2)
    dev[1, k + m - 1, S - 1] ^= 0x40
    dev[0, 0, 0] ^= 1
    # erase the worst case: first m shards (all data when m <= k)
    erased = list(range(min(m, k + m - k)))
    golden = dev.clone()
    dev[:, erased, :] = 0
    enc.reconstruct_batch(ptrs, S, nstripes, erased)
    assert torch.equal(dev[:, :, :S], golden[:, :, :S])


@pytest.mark.parametrize("size", [0, 1, 3, 4, 15, 16, 1023, 1024, 1025, 262144 + 5, 5592406])
def test_crc32_matches_oracle(rs, size):
    r = rng(size)
    arrs = [r.integers(0, 256, size, dtype=np.uint8) for _ in range(3)]
    d = [torch.from_numpy(a).cuda() if size else torch.zeros(1, dtype=torch.uint8, device="cuda") for a in arrs]
    got = rs.crc32_ieee_batch([t.data_ptr() for t in d], size)
    want = [O.crc32_ieee(a) for a in arrs]
    assert got == want


def test_crc32_known_answer(rs):
    t = torch.frombuffer(bytearray(b"123456789"), dtype=torch.uint8).cuda()
    assert rs.crc32_ieee_batch([t.data_ptr()], 9) == [0xCBF43926]


def test_large_stripe_roundtrip_ec12p4(rs):
    """BASELINE C2/C3 shape: 64 MiB blob -> S = 5,592,406.  Oracle-checked encode, then the
    size-independent property: erase {0,1,2,3} -> reconstruct -> identical stripe."""
    k, m, S = 12, 4, 5592406
    host, dev, ptrs, pitch = _stripe_batch(k, m, S, 2, seed=0xCF5EC000)
    enc = rs.New(k, m)
    enc.encode_batch(ptrs, S, 2)
    want = [host[0, i, :S].copy() for i in range(k + m)]
    assert O.encode(k, m, want) == 0
    got = dev[0, :, :S].cpu().numpy()
    for i in range(k, k + m):
        assert np.array_equal(got[i], want[i])
    golden = dev.clone()
    dev[:, 0:4, :] = 0
    enc.reconstruct_batch(ptrs, S, 2, [0, 1, 2, 3])
    assert torch.equal(dev[:, :, :S], golden[:, :, :S])
    flags = torch.zeros(2, dtype=torch.int32, device="cuda")
    enc.verify_batch(ptrs, S, 2, flags.data_ptr())
    assert flags.cpu().tolist() == [0, 0]


@pytest.mark.parametrize("k,m", [(8, 1), (12, 1), (6, 2), (3, 4), (10, 4), (12, 4), (16, 4)])
@pytest.mark.parametrize("size", [16, 17, 31, 4096 + 5, 65536 + 15, 174763])
def test_ragged_row_end_encode_verify_reconstruct(rs, k, m, size):
    """The fixed-K kernels code a row's ragged end as the last full 16-byte chunk of the row (the
    lane's bytes before the end repeat its neighbour's with the same values): encode equals the
    oracle to the last byte, Verify catches a flip in the last byte of any row (and in the first byte
    of the overlapped chunk), Reconstruct rebuilds the last bytes of lost rows."""
    want = oracle_encoded(k, m, size, seed=size * 7 + k)
    enc = engine(rs, k, m)
    d = to_dev([s if i < k else np.zeros(size, np.uint8) for i, s in enumerate(want)])
    enc.Encode(d)
    got = to_host(d)
    for i in range(k + m):
        assert np.array_equal(got[i], want[i]), (i, size)
    assert enc.Verify(to_dev(want))
    for idx in (k + m - 1, k, 0):
        for pos in (size - 1, max(0, size - 16)):
            bad = [s.copy() for s in want]
            bad[idx][pos] ^= 0x80
            assert not enc.Verify(to_dev(bad)), (idx, pos, size)
    for erased, data_only in (({0}, True), (set(range(min(m, k))), False), ({k - 1, k + m - 1} if m > 1 else {k}, False)):
        _check_recon(rs, k, m, size, erased, data_only, seed=size + len(erased))
