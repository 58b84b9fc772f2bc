"""Encode / reconstruct with fused shard checksums (cfsec_rs_{encode,reconstruct}_crc_batch).

CubeFS computes crc32.ChecksumIEEE of every shard right after Encode (access/stream_put.go:249-253)
and of repaired shards (blobnode/work_shard_recover.go:335-342).  The GPU computes them inside the
coding kernel; every word must equal zlib's CRC-32 (the same polynomial, preset and final inversion
as Go's hash/crc32 IEEE) of the shard bytes, and the coded bytes must still match the oracle.
Shapes outside the fused kernel's range (m > 6, k not a code-mode count) take the product + the
standalone CRC kernel and must give the same words.
"""
import zlib

import numpy as np
import pytest

from oracle import oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

# (12, 4) (8, 1) (16, 4) (6, 3) (8, 2) (16, 3) (12, 1): the lookup-product fused kernel (m <= 4, k <= 16);
# (6, 6) (18, 1): the v_perm fused kernels; (6, 10) (10, 4) (16, 20): product + standalone CRC
SHAPES = [(12, 4), (6, 6), (8, 1), (18, 1), (16, 4), (6, 10), (10, 4), (16, 20), (6, 3), (8, 2), (16, 3), (12, 1)]
SIZES = [1, 15, 16, 17, 4095, 4096, 4097, 8191, 65539, 174763]


@pytest.fixture(scope="module")
def rs():
    from chubaofs_amd import reedsolomon
    return reedsolomon


def crc(a: np.ndarray) -> int:
    return zlib.crc32(a.tobytes()) & 0xFFFFFFFF


def batch(k, m, S, nstripes, seed, pitch=None):
    total = k + m
    pitch = pitch or (S + 255) // 256 * 256
    r = np.random.default_rng(seed)
    host = np.zeros((nstripes, total, pitch), np.uint8)
    host[:, :k, :S] = r.integers(0, 256, (nstripes, k, S), dtype=np.uint8)
    dev = torch.from_numpy(host).cuda()
    base = dev.data_ptr()
    ptrs = [base + (s * total + i) * pitch for s in range(nstripes) for i in range(total)]
    return host, dev, ptrs


@pytest.mark.parametrize("k,m", SHAPES)
@pytest.mark.parametrize("S", SIZES)
def test_encode_crc_batch(rs, k, m, S):
    nst = 3
    host, dev, ptrs = batch(k, m, S, nst, seed=k * 100 + m + S)
    crcs = torch.full((nst * (k + m),), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    enc = rs.New(k, m)
    enc.encode_crc_batch(ptrs, S, nst, crcs.data_ptr())
    got = dev.cpu().numpy()
    words = crcs.cpu().numpy().view(np.uint32).reshape(nst, k + m)
    for s in range(nst):
        want = [host[s, i, :S].copy() for i in range(k + m)]
        assert O.encode(k, m, want) == 0
        for i in range(k + m):
            assert np.array_equal(got[s, i, :S], want[i]), (s, i)
            assert int(words[s, i]) == crc(want[i]), (s, i, hex(int(words[s, i])), hex(crc(want[i])))
            assert int(words[s, i]) == O.crc32_ieee(want[i])


@pytest.mark.parametrize("k,m,S", [(12, 4, 100003), (6, 6, 4097), (16, 4, 262144)])
def test_encode_crc_explicit_pointer_table(rs, k, m, S):
    """Shards in separate allocations (no common stripe stride): the pointer-table path."""
    nst = 5
    r = np.random.default_rng(S)
    shards = [[torch.from_numpy(r.integers(0, 256, S, dtype=np.uint8)).cuda() if i < k
               else torch.zeros(S, dtype=torch.uint8, device="cuda") for i in range(k + m)] for _ in range(nst)]
    ptrs = [t.data_ptr() for st in shards for t in st]
    crcs = torch.zeros(nst * (k + m), dtype=torch.int32, device="cuda")
    rs.New(k, m).encode_crc_batch(ptrs, S, nst, crcs.data_ptr())
    words = crcs.cpu().numpy().view(np.uint32).reshape(nst, k + m)
    for s in range(nst):
        want = [t.cpu().numpy() for t in shards[s]]
        host = [w.copy() for w in want]
        assert O.encode(k, m, host) == 0
        for i in range(k + m):
            assert np.array_equal(want[i], host[i])
            assert int(words[s, i]) == crc(host[i]), (s, i)


@pytest.mark.parametrize("k,m,erased", [(12, 4, [0, 1, 2, 3]), (12, 4, [3, 13]), (6, 6, [0, 5, 6, 11]),
                                        (8, 1, [4]), (18, 1, [17]), (16, 20, [0, 1, 16, 17]), (6, 10, [2, 9])])
@pytest.mark.parametrize("S", [17, 4096, 70001])
def test_reconstruct_crc_batch(rs, k, m, erased, S):
    nst = 4
    host, dev, ptrs = batch(k, m, S, nst, seed=S + len(erased))
    enc = rs.New(k, m)
    enc.encode_batch(ptrs, S, nst)
    golden = dev.clone()
    dev[:, erased, :] = 0
    crcs = torch.full((nst * (k + m),), -1, dtype=torch.int32, device="cuda")
    enc.reconstruct_crc_batch(ptrs, S, nst, erased, crcs.data_ptr())
    assert torch.equal(dev[:, :, :S], golden[:, :, :S])
    g = golden.cpu().numpy()
    words = crcs.cpu().numpy().view(np.uint32).reshape(nst, k + m)
    for s in range(nst):
        for i in range(k + m):
            want = crc(g[s, i, :S]) if i in erased else 0
            assert int(words[s, i]) == want, (s, i)


def test_crc_large_stripe_ec12p4(rs):
    """BASELINE C2 shape (S = 5,592,406): every shard's checksum after a fused encode, then the
    rebuilt shards' checksums after the worst-case reconstruct equal the originals'."""
    k, m, S, nst = 12, 4, 5592406, 2
    host, dev, ptrs = batch(k, m, S, nst, seed=0xCF5EC000)
    enc = rs.New(k, m)
    crcs = torch.zeros(nst * (k + m), dtype=torch.int32, device="cuda")
    enc.encode_crc_batch(ptrs, S, nst, crcs.data_ptr())
    g = dev.cpu().numpy()
    words = crcs.cpu().numpy().view(np.uint32).reshape(nst, k + m)
    for s in range(nst):
        for i in range(k + m):
            assert int(words[s, i]) == crc(g[s, i, :S]), (s, i)
    want = words.copy()
    dev[:, 0:4, :] = 0
    rc = torch.zeros_like(crcs)
    enc.reconstruct_crc_batch(ptrs, S, nst, [0, 1, 2, 3], rc.data_ptr())
    rw = rc.cpu().numpy().view(np.uint32).reshape(nst, k + m)
    assert (rw[:, :4] == want[:, :4]).all() and (rw[:, 4:] == 0).all()


def test_crc_zero_length_and_empty(rs):
    enc = rs.New(12, 4)
    crcs = torch.full((16,), 7, dtype=torch.int32, device="cuda")
    t = torch.zeros(16, dtype=torch.uint8, device="cuda")
    enc.encode_crc_batch([t.data_ptr()] * 16, 0, 1, crcs.data_ptr())
    assert crcs.cpu().tolist() == [0] * 16  # crc32.ChecksumIEEE(nil) == 0


@pytest.mark.parametrize("layout", ["pitched", "separate"])
@pytest.mark.parametrize("n,S", [(170, 4097), (2048, 300), (7, 349526)])
def test_standalone_crc_many_shards(rs, layout, n, S):
    """cfsec_crc32_ieee_batch over many shards: an equally spaced list runs as one launch, a
    scattered list in pointer-table launches of 160."""
    r = np.random.default_rng(n + S)
    if layout == "pitched":
        pitch = (S + 255) // 256 * 256
        host = r.integers(0, 256, (n, pitch), dtype=np.uint8)
        dev = torch.from_numpy(host).cuda()
        ptrs = [dev.data_ptr() + i * pitch for i in range(n)]
        arrs = [host[i, :S] for i in range(n)]
    else:
        arrs = [r.integers(0, 256, S, dtype=np.uint8) for _ in range(n)]
        dev = [torch.from_numpy(a).cuda() for a in arrs]
        ptrs = [t.data_ptr() for t in dev]
    assert rs.crc32_ieee_batch(ptrs, S) == [crc(a) for a in arrs]


@pytest.mark.parametrize("memory", ["pageable", "pinned", "device"])
@pytest.mark.parametrize("k,m,S", [(12, 4, 5592406), (12, 4, 17), (6, 6, 174763), (16, 20, 4097), (8, 1, 65536)])
def test_encode_crc_single_call(rs, memory, k, m, S):
    """cfsec_rs_encode_crc: the access Put path's Encode + per-shard ChecksumIEEE in one call, for
    Go-side host buffers (pageable or from cfsec_host_alloc) and device shards."""
    from chubaofs_amd import _lib
    r = np.random.default_rng(S + k)
    want = [r.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
    assert O.encode(k, m, want) == 0
    if memory == "device":
        sh = [torch.from_numpy(w.copy()).cuda() for w in want]
        for p in sh[k:]:
            p.zero_()
    else:
        buf = _lib.pinned_empty((k + m) * S) if memory == "pinned" else np.zeros((k + m) * S, np.uint8)
        sh = [buf[i * S:(i + 1) * S] for i in range(k + m)]
        for i in range(k):
            sh[i][:] = want[i]
    words = rs.New(k, m).EncodeCRC(sh)
    got = [s.cpu().numpy() if hasattr(s, "cpu") else s for s in sh]
    for i in range(k + m):
        assert np.array_equal(got[i], want[i]), i
        assert words[i] == crc(want[i]), i
