"""The bit-sliced fused kernel's remainder tiles (gf_bs_crc.hip, round 6): with tps = B W + r column
tiles per row, the W-strided rounds stop at B W and the r tiles of every stripe go one per wave of
extra workgroups, each folding its single tile into the row's checksum word on its own.  The shapes
here are put batches large enough that W < tps and r > 0 on a 256-CU MI355X (the launch trace, read
from CFSEC_TRACE_CRC, must show tail > 0): the C4 put (EC6P10L2, 48 bids), EC12P4 (3 waves per SIMD,
input registers in LDS), EC6P6L9 (output registers in LDS, 2 waves per SIMD) with and without the
checksums, the 16 + 20 code (both register sets in LDS) and EC3P3 (k odd: no paired basis), rows at
odd pitches (every row misaligned, the last tile partial).  Every bid's words equal zlib's CRC-32 of
the rows the call wrote, every bid's parity equals the engine's encode without checksums, and the
first and last bids' parity equals the ec oracle's Encode (lrcencoder.go:35-70 over KRS
reedsolomon.go:609-625, restated in oracle/ec_oracle.py)."""
import re
import zlib

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

CASES = [  # mode, bids, S
    ("EC6P10L2", 48, 699051),
    ("EC12P4", 24, 699051),
    ("EC6P6L9", 32, 699051),
    ("EC16P20L2", 16, 300001),
    ("EC3P3", 128, 100003),
]


def _tails(err: str):
    return [int(t) for t in re.findall(r"cfsec: bs launch .* tail=(\d+)", err)]


@pytest.mark.parametrize("mode,nb,S", CASES)
def test_tail_waves_put_batch(mode, nb, S, monkeypatch, capfd):
    from chubaofs_amd import codemode as cm, ec
    from oracle.ec_oracle import ECOracle, Slice
    t = cm.GetTactic(getattr(cm, mode))
    total = t.N + t.M + t.L
    enc = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=False), device=0)
    g = torch.Generator(device="cuda").manual_seed(S + nb)
    buf = torch.zeros((nb, total, S), dtype=torch.uint8, device="cuda")
    buf[:, :t.N] = torch.randint(0, 256, (nb, t.N, S), dtype=torch.uint8, device="cuda", generator=g)
    plain = buf.clone()
    # the engine's encode without checksums (for EC6P6L9 the bit-sliced plain route, its tails too)
    monkeypatch.setenv("CFSEC_TRACE_CRC", "1")
    capfd.readouterr()
    st = enc.EncodeBatch([[plain[b, i] for i in range(total)] for b in range(nb)])
    torch.cuda.synchronize()
    err_plain = capfd.readouterr().err
    assert st == [0] * nb
    if mode == "EC6P6L9":
        assert "bs plain" in err_plain and any(_tails(err_plain)), err_plain[-2000:]
    st, crcs = enc.EncodeBatch([[buf[b, i] for i in range(total)] for b in range(nb)], crcs=True)
    torch.cuda.synchronize()
    err = capfd.readouterr().err
    assert st == [0] * nb
    assert "bs crc" in err and any(_tails(err)), err[-2000:]
    assert torch.equal(buf, plain)
    got = buf.cpu().numpy()
    for b in range(nb):
        for i in range(total):
            assert crcs[b][i] == zlib.crc32(got[b, i].tobytes()) & 0xFFFFFFFF, (b, i)
    orc = ECOracle.from_tactic(t, enable_verify=False)
    for b in (0, nb - 1):
        ref = [Slice.of(got[b, i].copy()) for i in range(t.N)] + [Slice.of(np.zeros(S, np.uint8)) for _ in range(total - t.N)]
        assert orc.encode(ref) == 0
        for i in range(t.N, total):
            assert np.array_equal(got[b, i], ref[i].view()), (b, i)


def test_tail_waves_pointer_table_launches(monkeypatch, capfd):
    """Shards in separate allocations (pointer-table launches of 96 / 16 = 6 stripes, the last one
    short) at BASELINE C2's row length, so W < tps in the full launches and the tail waves run there:
    13 EC12P4 stripes through encode_crc_batch, parity vs the plain encode and the C oracle (first and
    last stripe), every word vs zlib."""
    from chubaofs_amd import reedsolomon
    from oracle import oracle as O
    k, m, S, nst = 12, 4, 5592406, 13
    g = torch.Generator(device="cuda").manual_seed(0x7A11)
    sh = [[torch.randint(0, 256, (S,), dtype=torch.uint8, device="cuda", generator=g) if i < k
           else torch.zeros(S, dtype=torch.uint8, device="cuda") for i in range(k + m)] for _ in range(nst)]
    ptrs = [t.data_ptr() for st in sh for t in st]
    enc = reedsolomon.New(k, m)
    monkeypatch.setenv("CFSEC_TRACE_CRC", "1")
    crcs = torch.zeros(nst * (k + m), dtype=torch.int32, device="cuda")
    capfd.readouterr()
    enc.encode_crc_batch(ptrs, S, nst, crcs.data_ptr())
    torch.cuda.synchronize()
    err = capfd.readouterr().err
    tails = _tails(err)
    # 6 + 6 + 1 stripes: the two full launches have W = 512 < tps = 2731 (171 tail tiles per stripe),
    # the lone stripe's launch W = tps
    assert "bs crc" in err and len(tails) == 3 and all(tails[:2]) and tails[2] == 0, err[-2000:]
    fused = [[t.cpu().numpy() for t in st] for st in sh]
    for st in sh:
        for t in st[k:]:
            t.zero_()
    enc.encode_batch(ptrs, S, nst)
    torch.cuda.synchronize()
    words = crcs.cpu().numpy().view(np.uint32).reshape(nst, k + m)
    for s_ in range(nst):
        for i in range(k + m):
            assert np.array_equal(fused[s_][i], sh[s_][i].cpu().numpy()), (s_, i)
            assert int(words[s_][i]) == zlib.crc32(fused[s_][i].tobytes()) & 0xFFFFFFFF, (s_, i)
    for s_ in (0, nst - 1):
        want = [fused[s_][i].copy() for i in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
        assert O.encode(k, m, want) == 0
        for i in range(k, k + m):
            assert np.array_equal(fused[s_][i], want[i]), (s_, i)
