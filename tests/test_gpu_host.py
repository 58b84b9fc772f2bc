"""Host-memory calls (CFSEC_MEM_HOST, what the cgo shim uses) through the chunked two-stream
pipeline: shards larger than one chunk (1 MiB per row), pageable and pinned (cfsec_host_alloc)
buffers, shards carved from one buffer at stride S (ec.Buffer, common/ec/buf.go:83-84: the 2-D
copy path) and separate buffers (per-row copies).  Bytes must match the oracle exactly."""
import numpy as np
import pytest

from chubaofs_amd import _lib
from oracle import oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def rs():
    from chubaofs_amd import reedsolomon
    return reedsolomon


def alloc(n, pinned):
    return _lib.pinned_empty(n) if pinned else np.zeros(n, np.uint8)


def make(k, m, S, pinned, contiguous, seed):
    r = np.random.default_rng(seed)
    if contiguous:
        buf = alloc((k + m) * S, pinned)
        buf[:k * S] = r.integers(0, 256, k * S, dtype=np.uint8)
        buf[k * S:] = 0
        return [buf[i * S:(i + 1) * S] for i in range(k + m)]
    out = []
    for i in range(k + m):
        a = alloc(S, pinned)
        a[:] = r.integers(0, 256, S, dtype=np.uint8) if i < k else 0
        out.append(a)
    return out


@pytest.mark.parametrize("pinned", [False, True])
@pytest.mark.parametrize("contiguous", [False, True])
@pytest.mark.parametrize("k,m,S", [(12, 4, 3 * (1 << 20) + 12345), (6, 6, (1 << 20) + 1), (16, 20, 2 * (1 << 20) + 256)])
def test_host_pipeline_encode_verify_reconstruct(pinned, contiguous, k, m, S):
    sh = make(k, m, S, pinned, contiguous, seed=S + k)
    want = [s.copy() for s in sh]
    assert O.encode(k, m, want) == 0
    enc = rs().New(k, m)
    enc.Encode(sh)
    for i in range(k + m):
        assert np.array_equal(sh[i], want[i]), i
    assert enc.Verify(sh)
    sh[k + m - 1][S - 1] ^= 1  # last byte of the last chunk
    assert not enc.Verify(sh)
    sh[k + m - 1][S - 1] ^= 1
    pos = min(S - 1, (1 << 20) + 7)  # second chunk of a data row
    sh[0][pos] ^= 0x80
    assert not enc.Verify(sh)
    sh[0][pos] ^= 0x80
    erased = list(range(min(m, 4)))
    work = [s[:0] if i in erased else s for i, s in enumerate(sh)]  # missing: len 0
    enc.Reconstruct(work)
    assert all(len(w) == S for w in work)
    for i in range(k + m):
        assert np.array_equal(work[i], want[i]), i
    # ec.Encoder style: the bad shards keep their (possibly pinned) buffers, rebuilt in place
    from chubaofs_amd import ec, codemode as cm
    if (k, m) == (12, 4):
        e = ec.NewEncoder(ec.Config(CodeMode=cm.GetTactic(cm.EC12P4), EnableVerify=True))
        for i in erased:
            sh[i][:] = 0
        e.Reconstruct(sh, erased)
        for i in range(k + m):
            assert np.array_equal(sh[i], want[i]), i


def test_pinned_alloc_roundtrip():
    a = _lib.pinned_empty(1 << 20)
    a[:] = 7
    assert int(a.sum()) == 7 << 20
    assert _lib.pinned_empty(0).size == 0


@pytest.mark.parametrize("k,m", [(12, 4), (6, 6)])
@pytest.mark.parametrize("delta", [-1, 0, 1])
def test_small_pageable_staging_boundary(k, m, delta):
    """Pageable host calls moving at most 1 MiB (rows x S) are copied into page-locked staging on the
    CPU and coded there (round 6: a degraded range read's segments, ~130 -> ~20 us); one byte more per
    row takes the chunked pipeline.  Encode, Verify (a flipped byte caught), ReconstructData and
    Reconstruct at both sides of the boundary, bytes equal to the oracle."""
    S = (1 << 20) // (k + m) + delta
    sh = make(k, m, S, False, False, seed=S * 3 + k)
    want = [s.copy() for s in sh]
    assert O.encode(k, m, want) == 0
    enc = rs().New(k, m)
    enc.Encode(sh)
    for i in range(k + m):
        assert np.array_equal(sh[i], want[i]), i
    assert enc.Verify(sh)
    sh[k][S // 2] ^= 0x10
    assert not enc.Verify(sh)
    sh[k][S // 2] ^= 0x10
    work = [s[:0] if i in (0, 1) else s.copy() for i, s in enumerate(sh)]
    enc.ReconstructData(work)
    assert np.array_equal(work[0], want[0]) and np.array_equal(work[1], want[1])
    work = [s[:0] if i in (1, k) else s.copy() for i, s in enumerate(sh)]
    enc.Reconstruct(work)
    for i in range(k + m):
        assert np.array_equal(work[i], want[i]), i
