"""Stream ordering of the C ABI (include/cfsec.h "Memory"): a call must never read its device input
before the kernel that produced it ran.

- stream=None in the Python binding means PyTorch's current stream of the buffers' device, so an
  input produced under `torch.cuda.stream(side)` (a non-blocking side stream) is ordered;
- a NULL hipStream_t in the C ABI orders the call after the legacy default stream with an event
  (the engine's own streams are non-blocking), which is what a C / cgo caller gets.

Each producer is delayed behind a long device sleep so that a missing dependency shows as stale
(zero) input rather than passing by luck.
"""
import zlib

import numpy as np
import pytest

from oracle import oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

K, M, S = 12, 4, 1 << 20
SLEEP_CYCLES = 50_000_000  # ~20 ms at 2.4 GHz


def _delay():
    if hasattr(torch.cuda, "_sleep"):
        torch.cuda._sleep(SLEEP_CYCLES)


def _want(h):
    shards = [h[i].copy() for i in range(K)] + [np.zeros(S, np.uint8) for _ in range(M)]
    assert O.encode(K, M, shards) == 0
    return shards[K:]


def _host(seed):
    return np.random.default_rng(seed).integers(0, 256, (K, S), dtype=np.uint8)


def test_encode_input_from_side_stream():
    from chubaofs_amd import reedsolomon
    enc = reedsolomon.New(K, M, device=0)
    h = _host(1)
    src = torch.from_numpy(h).cuda()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    buf = torch.zeros((K + M, S), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        _delay()
        buf[:K].copy_(src)          # the producer, queued behind the sleep on the side stream
        enc.Encode([buf[i] for i in range(K + M)])  # stream=None: the side stream
    torch.cuda.synchronize()
    want = _want(h)
    got = buf[K:].cpu().numpy()
    for r in range(M):
        assert np.array_equal(got[r], want[r]), r


def test_encode_batch_input_from_side_stream():
    from chubaofs_amd import reedsolomon
    enc = reedsolomon.New(K, M, device=0)
    nst = 3
    hs = [_host(10 + s) for s in range(nst)]
    src = torch.from_numpy(np.stack(hs)).cuda()
    buf = torch.zeros((nst, K + M, S), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    ptrs = [buf[s, i].data_ptr() for s in range(nst) for i in range(K + M)]
    with torch.cuda.stream(side):
        _delay()
        buf[:, :K].copy_(src)
        enc.encode_batch(ptrs, S, nst)  # stream=None: the side stream
        crcs = torch.zeros(nst * (K + M), dtype=torch.int32, device="cuda")
        enc.encode_crc_batch(ptrs, S, nst, crcs.data_ptr())
    torch.cuda.synchronize()
    words = crcs.cpu().numpy().view(np.uint32)
    for s in range(nst):
        want = _want(hs[s])
        got = buf[s, K:].cpu().numpy()
        for r in range(M):
            assert np.array_equal(got[r], want[r]), (s, r)
        for i in range(K + M):
            row = hs[s][i] if i < K else want[i - K]
            assert int(words[s * (K + M) + i]) == zlib.crc32(row.tobytes()) & 0xFFFFFFFF


def test_crc32block_encode_input_from_side_stream():
    from chubaofs_amd import crc32block as C
    h = np.random.default_rng(3).integers(0, 256, S, dtype=np.uint8)
    src = torch.from_numpy(h).cuda()
    buf = torch.zeros(S, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        _delay()
        buf.copy_(src)
        framed, crc = C.Encode(buf)
    torch.cuda.synchronize()
    assert crc == zlib.crc32(h.tobytes()) & 0xFFFFFFFF
    assert np.array_equal(framed.cpu().numpy(), O.crc32block_encode(h))


def test_null_stream_orders_after_default_stream():
    """A C caller's NULL stream: the input written on the legacy default stream is seen."""
    from chubaofs_amd import _lib, reedsolomon
    enc = reedsolomon.New(K, M, device=0)
    h = _host(4)
    src = torch.from_numpy(h).cuda()
    buf = torch.zeros((K + M, S), dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    assert torch.cuda.current_stream().cuda_stream == 0  # PyTorch's default stream is the null stream
    _delay()
    buf[:K].copy_(src)  # on the null stream, behind the sleep
    shards = [buf[i] for i in range(K + M)]
    from chubaofs_amd._shards import Marshal
    m = Marshal(shards)
    _lib.check(_lib.lib().cfsec_rs_encode(enc._h, m.ptr(), m.n, m.mem, None))  # explicit NULL stream
    want = _want(h)
    got = buf[K:].cpu().numpy()
    for r in range(M):
        assert np.array_equal(got[r], want[r]), r
