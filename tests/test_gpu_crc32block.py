"""crc32block framing on the GPU (cfsec_crc32block_encode / _decode) against the oracle.

Every framed byte must equal the oracle's (oracle.crc32block_encode: encode.go:87-109 +
block.go:46-49), the whole-shard checksum must equal crc32.ChecksumIEEE of the payload (zlib),
and Decoder.Reader ranges (encode_test.go:76-93, :178-199) must read back the payload with every
touched block checked.
"""
import zlib

import numpy as np
import pytest

from oracle import oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

K = 1024
FSIZE = 128 * K + 80
SIZES = [1, 15, 16, 17, 4095, 4096, 4097, 64 * K - 5, 64 * K - 4, 64 * K, 64 * K + 4, FSIZE, 1 << 20, 5592406]
# encode_test.go:76-93 (TestDecodeData) on fsize = 128 KiB + 80
RANGES = [(0, 0), (FSIZE, FSIZE), (0, FSIZE), (64 * K - 4, FSIZE), (64 * K, FSIZE), (64 * K + 4, FSIZE),
          (64 * K + 5, FSIZE), (64 * K - 4, FSIZE - 1), (64 * K, FSIZE - 1), (64 * K + 4, FSIZE - 1),
          (64 * K + 5, FSIZE - 1), (64 * K + 4, FSIZE - 64 * K), (64 * K + 4, FSIZE - 64 * K - 4),
          (64 * K + 4, FSIZE - 64 * K - 5), (0, FSIZE - 64 * K - 4 - 64 * K - 4), (0, 64)]
# encode_test.go:178-199 (TestLimitEncoderReader2): (fsize, from, to)
RANGES2 = [(1, 0, 1), (64 * K - 4, 0, 64), (64 * K - 4, 0, 64 * K - 4), (64 * K, 0, 64 * K - 4), (64 * K, 0, 64 * K),
           (64 * K + 5, 0, 64 * K), (128 * K, 0, 128 * K), (128 * K, 128 * K - 4, 128 * K),
           (128 * K, 64 * K - 4, 64 * K), (128 * K, 64 * K + 4, 64 * K + 4), (128 * K, 64 * K + 4, 64 * K + 8),
           (128 * K, 64 * K + 7, 64 * K + 10), (128 * K, 64 * K - 4, 64 * K - 1), (128 * K, 4, 64 * K - 1),
           (128 * K, 4, 64 * K - 4), (128 * K, 4, 64 * K), (128 * K, 64 * K, 128 * K), (128 * K + 7, 64 * K, 64 * K),
           (128 * K + 7, 64 * K + 4, 128 * K), (128 * K + 7, 64 * K - 4, 128 * K + 7)]


@pytest.fixture(scope="module")
def C():
    from chubaofs_amd import crc32block
    return crc32block


def data(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8)


@pytest.mark.parametrize("size", SIZES)
@pytest.mark.parametrize("block_len", [4096, 64 * K, 1 << 20])
def test_encode_matches_oracle_device(C, size, block_len):
    d = data(size, size ^ block_len)
    framed, crc = C.Encode(torch.from_numpy(d).cuda(), block_len=block_len)
    want = O.crc32block_encode(d, block_len)
    assert np.array_equal(framed.cpu().numpy(), want)
    assert crc == zlib.crc32(d.tobytes()) & 0xFFFFFFFF


@pytest.mark.parametrize("memory", ["pageable", "pinned"])
@pytest.mark.parametrize("size", [1, 64 * K + 4, FSIZE, 5592406])
def test_encode_host_memory(C, memory, size):
    from chubaofs_amd import _lib
    d = data(size, size)
    src = _lib.pinned_empty(size) if memory == "pinned" else np.empty(size, np.uint8)
    src[:] = d
    dst = _lib.pinned_empty(C.EncodeSize(size)) if memory == "pinned" else None
    framed, crc = C.Encode(src, dst=dst)
    assert np.array_equal(framed, O.crc32block_encode(d))
    assert crc == zlib.crc32(d.tobytes()) & 0xFFFFFFFF


def test_encode_empty(C):
    framed, crc = C.Encode(torch.zeros(0, dtype=torch.uint8, device="cuda"))
    assert framed.numel() == 0 and crc == 0


@pytest.mark.parametrize("lo,hi", RANGES)
def test_decode_ranges(C, lo, hi):
    d = data(FSIZE, 11)
    framed = torch.from_numpy(O.crc32block_encode(d)).cuda()
    got = C.Decode(framed, FSIZE, lo, hi)
    assert np.array_equal(got.cpu().numpy(), d[lo:hi])


@pytest.mark.parametrize("fsize,lo,hi", RANGES2)
def test_decode_ranges_limit_encoder(C, fsize, lo, hi):
    d = data(fsize, fsize + lo)
    framed, _ = C.Encode(torch.from_numpy(d).cuda())  # GPU-framed, GPU-decoded
    got = C.Decode(framed, fsize, lo, hi)
    assert np.array_equal(got.cpu().numpy(), d[lo:hi])


@pytest.mark.parametrize("memory", ["pageable", "pinned"])
def test_decode_host_memory(C, memory):
    from chubaofs_amd import _lib
    d = data(FSIZE, 3)
    f = O.crc32block_encode(d)
    src = _lib.pinned_empty(f.size) if memory == "pinned" else np.empty(f.size, np.uint8)
    src[:] = f
    dst = _lib.pinned_empty(FSIZE) if memory == "pinned" else None
    assert np.array_equal(C.Decode(src, FSIZE, 0, FSIZE, dst=dst)[:FSIZE], d)
    assert np.array_equal(C.Decode(src, FSIZE, 64 * K + 5, FSIZE - 1), d[64 * K + 5:FSIZE - 1])


@pytest.mark.parametrize("where", ["payload", "header", "last"])
def test_decode_detects_corruption(C, where):
    from chubaofs_amd import _lib
    size = 5 * (64 * K - 4) + 1000  # 6 blocks
    d = data(size, 5)
    f = O.crc32block_encode(d)
    blk = {"payload": 2, "header": 3, "last": 5}[where]
    pos = blk * 64 * K + (1 if where == "header" else 4 + 777 % (size - blk * (64 * K - 4)))
    f[pos] ^= 0x20
    framed = torch.from_numpy(f).cuda()
    with pytest.raises(_lib.ErrMismatchedCrc) as ei:
        C.Decode(framed, size, 0, size)
    assert ei.value.block == blk
    with pytest.raises(_lib.ErrMismatchedCrc) as ei:
        C.Decode(framed, size, blk * (64 * K - 4) + 3, blk * (64 * K - 4) + 3)  # from == to inside it
    assert ei.value.block == blk
    # ranges that stay clear of the block read back fine
    lo, hi = (0, blk * (64 * K - 4)) if blk else (64 * K, size)
    assert np.array_equal(C.Decode(framed, size, lo, hi).cpu().numpy(), d[lo:hi])
    want = O.crc32block_decode(f, size, 0, size)[1]
    assert want == blk


def test_large_roundtrip_and_shard_crc(C):
    """A 64 MiB payload (1025 blocks): framed bytes, the whole-shard checksum and the round trip."""
    size = 64 << 20
    g = torch.Generator(device="cuda")
    g.manual_seed(0xCF5EC000)
    d = torch.randint(0, 256, (size,), generator=g, device="cuda", dtype=torch.uint8)
    framed, crc = C.Encode(d)
    h = d.cpu().numpy()
    assert crc == zlib.crc32(h.tobytes()) & 0xFFFFFFFF
    assert np.array_equal(framed.cpu().numpy(), O.crc32block_encode(h))
    back = C.Decode(framed, size)
    assert torch.equal(back, d)


@pytest.mark.parametrize("n,size", [(1, 1), (3, 64 * K - 4), (16, 349526), (130, 4097)])
def test_batch_encode_decode(C, n, size):
    """cfsec_crc32block_{encode,decode}_batch: n objects of one size (> 96 spans launches)."""
    framed_len = C.EncodeSize(size)
    g = torch.Generator(device="cuda")
    g.manual_seed(n * 1000 + size)
    src = torch.randint(0, 256, (n, size), generator=g, device="cuda", dtype=torch.uint8)
    dst = torch.full((n, framed_len), 0xEE, dtype=torch.uint8, device="cuda")
    crcs = torch.full((n,), 7, dtype=torch.int32, device="cuda")
    C.encode_batch([src[i].data_ptr() for i in range(n)], [dst[i].data_ptr() for i in range(n)], size,
                   shard_crcs_ptr=crcs.data_ptr())
    h, f = src.cpu().numpy(), dst.cpu().numpy()
    words = crcs.cpu().numpy().view(np.uint32)
    for i in range(n):
        assert np.array_equal(f[i], O.crc32block_encode(h[i])), i
        assert int(words[i]) == zlib.crc32(h[i].tobytes()) & 0xFFFFFFFF, i
    # corrupt object n-1's last block, then decode everything back
    dst[n - 1, framed_len - 1] ^= 1
    back = torch.zeros_like(src)
    bad = torch.zeros(n, dtype=torch.int32, device="cuda")
    C.decode_batch([dst[i].data_ptr() for i in range(n)], [back[i].data_ptr() for i in range(n)], size,
                   bad.data_ptr())
    b = bad.cpu().numpy().view(np.uint32)
    nblk = (size + 64 * K - 5) // (64 * K - 4)
    assert list(b[:-1]) == [0xFFFFFFFF] * (n - 1) and int(b[-1]) == nblk - 1
    assert torch.equal(back[:-1], src[:-1])


@pytest.mark.parametrize("doff", [0, 1, 4, 60, 127])
@pytest.mark.parametrize("block_len", [4096, 64 * K])
def test_decode_destination_alignment(C, doff, block_len):
    """Decode writes consecutive blocks' payloads back to back; the 128-byte line across each seam
    has one writer (crc32block.hip).  Every destination alignment, whole objects and a sub-range:
    the payload bytes, and no byte written outside [dst, dst + to - from)."""
    size = 7 * (block_len - 4) + 333
    d = data(size, doff + block_len)
    framed = torch.from_numpy(O.crc32block_encode(d, block_len)).cuda()
    n = 3
    for lo, hi in [(0, size), (block_len + 3, 5 * (block_len - 4) + 17), (size - 100, size)]:
        buf = torch.full((n, size + 256), 0xA5, dtype=torch.uint8, device="cuda")
        bad = torch.zeros(n, dtype=torch.int32, device="cuda")
        C.decode_batch([framed.data_ptr()] * n, [buf[i].data_ptr() + doff for i in range(n)], size, bad.data_ptr(),
                       from_=lo, to=hi, block_len=block_len)
        assert (bad.cpu().numpy().view(np.uint32) == 0xFFFFFFFF).all()
        h = buf.cpu().numpy()
        for i in range(n):
            assert np.array_equal(h[i, doff:doff + hi - lo], d[lo:hi]), (i, lo, hi)
            assert (h[i, :doff] == 0xA5).all() and (h[i, doff + hi - lo:] == 0xA5).all(), (i, lo, hi)
