"""crc32block framing (blobstore/common/crc32block) -- CPU side: the oracle restatement against the
reference's own vectors, and the C ABI's host-only size functions.

Pinning: EncodeSize / DecodeSize and the invalid block lengths are the literal vectors of
util_test.go:23-63; the block checksum is crc32.ChecksumIEEE (pinned by the 0xCBF43926 check value
in test_oracle.py); the framing itself follows encode.go:87-109 / block.go:46-49 and is checked
here against an independent zlib-based reading of the format.
"""
import zlib

import numpy as np
import pytest

from oracle import oracle as O

# util_test.go:29-31 (TestDecodeSize) and :54-56 (TestSetBlockSize): (blockLen, fsize, encodeSize)
SIZE_VECTORS = [(64 * 1024, 1, 5), (64 * 1024, 64 * 1024 - 4, 64 * 1024), (64 * 1024, 64 * 1024, 64 * 1024 + 8),
                (1 << 12, 1, 5), (1 << 20, 64 * 1024 - 4, 64 * 1024)]
INVALID_BLOCK_LENS = [-100, -1, 0, 4096 - 1, 4096 + 1]  # util_test.go:41

# encode_test.go:76-93 (TestDecodeData) with fsize = 128 KiB + 80
K = 1024
FSIZE = 128 * K + 80
RANGES = [(0, 0), (FSIZE, FSIZE), (0, FSIZE), (64 * K - 4, FSIZE), (64 * K, FSIZE), (64 * K + 4, FSIZE),
          (64 * K + 5, FSIZE), (64 * K - 4, FSIZE - 1), (64 * K, FSIZE - 1), (64 * K + 4, FSIZE - 1),
          (64 * K + 5, FSIZE - 1), (64 * K + 4, FSIZE - 64 * K), (64 * K + 4, FSIZE - 64 * K - 4),
          (64 * K + 4, FSIZE - 64 * K - 5), (0, FSIZE - 64 * K - 4 - 64 * K - 4), (0, 64)]


@pytest.mark.parametrize("block_len,fsize,enc", SIZE_VECTORS)
def test_oracle_sizes_match_reference_vectors(block_len, fsize, enc):
    assert O.crc32block_encode_size(fsize, block_len) == enc
    assert O.crc32block_decode_size(enc, block_len) == fsize


@pytest.mark.parametrize("block_len,fsize,enc", SIZE_VECTORS)
def test_cabi_sizes_match_reference_vectors(block_len, fsize, enc):
    from chubaofs_amd import crc32block as C
    assert C.EncodeSize(fsize, block_len) == enc
    assert C.DecodeSize(enc, block_len) == fsize


@pytest.mark.parametrize("block_len", INVALID_BLOCK_LENS)
def test_invalid_block_len(block_len):
    from chubaofs_amd import _lib
    from chubaofs_amd import crc32block as C
    with pytest.raises(ValueError):
        O.crc32block_encode_size(10, block_len)
    with pytest.raises(_lib.ErrInvalidBlock):
        C.EncodeSize(10, block_len)
    with pytest.raises(_lib.ErrInvalidBlock):
        C.DecodeSize(10, block_len)
    # the device entry points refuse the length before touching memory or the GPU
    assert _lib.lib().cfsec_crc32block_encode(None, 0, block_len, None, None, _lib.MEM_HOST, -1, None) == \
        _lib.ErrInvalidBlock.status


def _zlib_frames(payload, block_len):
    P = block_len - 4
    out = b""
    for q in range(0, len(payload), P):
        piece = payload[q:q + P]
        out += (zlib.crc32(piece) & 0xFFFFFFFF).to_bytes(4, "little") + piece
    return out


@pytest.mark.parametrize("size", [0, 1, 64 * K - 5, 64 * K - 4, 64 * K, 64 * K + 4, FSIZE, 1 << 20])
@pytest.mark.parametrize("block_len", [4096, 64 * K, 1 << 20])
def test_oracle_encode_layout(size, block_len):
    d = np.random.default_rng(size + block_len).integers(0, 256, size, dtype=np.uint8)
    f = O.crc32block_encode(d, block_len)
    assert f.size == O.crc32block_encode_size(size, block_len)
    assert f.tobytes() == _zlib_frames(d.tobytes(), block_len)


@pytest.mark.parametrize("lo,hi", RANGES)
def test_oracle_decode_ranges(lo, hi):
    """encode_test.go TestDecodeData: every range reads back data[from:to]."""
    d = np.random.default_rng(7).integers(0, 256, FSIZE, dtype=np.uint8)
    f = O.crc32block_encode(d)
    got, bad = O.crc32block_decode(f, FSIZE, lo, hi)
    assert bad == -1 and np.array_equal(got, d[lo:hi])


def test_oracle_decode_detects_corruption():
    d = np.random.default_rng(8).integers(0, 256, FSIZE, dtype=np.uint8)
    f = O.crc32block_encode(d)
    f[64 * K + 100] ^= 1  # payload of block 1
    assert O.crc32block_decode(f, FSIZE, 0, 10)[1] == -1          # block 0 only
    assert O.crc32block_decode(f, FSIZE, 0, 64 * K)[1] == 1       # reaches block 1
    assert O.crc32block_decode(f, FSIZE, 64 * K + 4, 64 * K + 4)[1] == 1  # from == to skips into block 1


@pytest.mark.parametrize("lo,hi", [(0, FSIZE), (64 * K + 4, FSIZE), (FSIZE - 1, FSIZE), (64 * K, 64 * K), (0, 10)])
def test_decode_short_source_is_short_data(lo, hi):
    """A framed object that ends before the last block [lo, hi) touches is refused before anything
    is read or copied (the reference's SectionReader gives io.ErrUnexpectedEOF, decode.go:94-97,
    126-130): host call, no device needed -- the check runs first."""
    from chubaofs_amd import _lib
    from chubaofs_amd import crc32block as C
    d = np.random.default_rng(9).integers(0, 256, FSIZE, dtype=np.uint8)
    f = O.crc32block_encode(d)
    P = 64 * K - 4
    last = (hi - 1) // P if lo < hi else lo // P  # from == to inside a block checks that block
    end = min(f.size, (last + 1) * 64 * K)       # framed end of the last touched block
    with pytest.raises(_lib.ErrShortData):
        C.Decode(np.ascontiguousarray(f[:end - 1]), FSIZE, lo, hi)


def test_decode_batch_short_source_is_short_data():
    from chubaofs_amd import _lib
    from chubaofs_amd import crc32block as C
    size = 3 * (64 * K - 4) + 10
    fake = [0x1000, 0x2000]  # never dereferenced: the length check comes first
    with pytest.raises(_lib.ErrShortData):
        C.decode_batch(fake, fake, size, 0x3000, src_len=C.EncodeSize(size) - 1)
    with pytest.raises(_lib.ErrShortData):  # only block 0 is touched, and it is cut
        C.decode_batch(fake, fake, size, 0x3000, 0, 10, src_len=64 * K - 1)
