"""Fused encode + every shard's crc32.ChecksumIEEE on the bit-sliced networks (gf_bs_crc.hip, round 6).

access checksums every data and parity shard right after Encode (blobstore/access/stream_put.go:
249-253).  For EC12P4 and EC6P10L2's fused LRC encode the product now runs as the bit-sliced XOR
network and every checksum comes from the bit planes it holds (56 lookups per lane and row, no row
re-read), W waves per stripe on every W-th tile, each folding its lanes' Horner registers once.  Checked here against the C oracle's Encode (KRS/reedsolomon.go:707-738 restated) and zlib's
CRC-32 at lengths around the 2 KiB column tile (a partial last tile, tiles shorter than a lane's
piece, lengths below 16), with rows at odd byte offsets, stripes in one allocation (one affine launch)
and in separate allocations (pointer-table launches), and with checksum words at a stride and slots
of the caller's choosing (the ec batch seam).  CFSEC_TRACE_CRC names the launches, so each case also
asserts that the bit-sliced route ran.

EC6P10L2's, the 16 + 20 code's (EC16P20, EC16P20L2) and the other modes' routes (EC6P8, EC6P10,
EC12P9, EC15P12, EC10P4, EC4P4, EC3P3 and the LRC modes EC6P3L3, EC4P4L2, EC6P6L9, EC6P8L10:
CFSEC_BS_CRC bits 0, 2, 4) and EC12P4's (bit 1, or bit 3) are on by default; a child process re-runs
the module with CFSEC_BS_CRC=253 (EC12P4 through bit 3, EC6P3's route on too).  The wide LRC modes' plain encodes (EC6P6L9, EC6P8L10) take the same
kernel without the checksums (bit 5, on).
"""
import os
import subprocess
import sys
import zlib

import numpy as np
import pytest

from oracle import oracle as O

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

SIZES = [1, 15, 16, 17, 1023, 1024, 1025, 2047, 2048, 2049, 4095, 4097, 6144, 65539, 174763]
MASK = int(os.environ.get("CFSEC_BS_CRC", "119"), 0)  # the library default
ec12p4 = pytest.mark.skipif(not MASK & 10, reason="EC12P4's route is off (CFSEC_BS_CRC without bits 1, 3)")
ec12p4_long = ec12p4
plain = pytest.mark.skipif(not MASK & 32, reason="the wide LRC modes' plain route is off (CFSEC_BS_CRC without bit 5)")
rs_more = pytest.mark.skipif(not MASK & 16, reason="the other RS modes' route is off (CFSEC_BS_CRC without bit 4)")
ec16 = pytest.mark.skipif(not MASK & 4, reason="the 16 + 20 code's route is off (CFSEC_BS_CRC without bit 2)")


@pytest.fixture(scope="module")
def rs():
    from chubaofs_amd import reedsolomon
    return reedsolomon


def crc(a: np.ndarray) -> int:
    return zlib.crc32(np.ascontiguousarray(a).tobytes()) & 0xFFFFFFFF


def routed(err: str, k: int, m: int) -> bool:
    return f"bs crc k={k} m={m}" in err


def check_stripes(k, m, host_rows, got_rows, words):
    for s, rows in enumerate(host_rows):
        want = [r.copy() for r in rows]
        assert O.encode(k, m, want) == 0
        for i in range(k + m):
            assert np.array_equal(got_rows[s][i], want[i]), (s, i)
            assert int(words[s][i]) == crc(want[i]), (s, i, hex(int(words[s][i])), hex(crc(want[i])))


@ec12p4
@pytest.mark.parametrize("S", SIZES)
@pytest.mark.parametrize("offset", [0, 3])
def test_ec12p4_encode_crc_affine(rs, S, offset, monkeypatch, capfd):
    """EC12P4 encode_crc_batch over 5 stripes in one allocation, rows at pitch S + offset (odd
    offsets: every row misaligned), one launch."""
    monkeypatch.setenv("CFSEC_TRACE_CRC", "1")
    k, m, nst = 12, 4, 5
    pitch = S + offset
    r = np.random.default_rng(S * 7 + offset)
    flat = np.zeros(nst * (k + m) * pitch + 64, np.uint8)
    rows = [[None] * (k + m) for _ in range(nst)]
    for s in range(nst):
        for i in range(k):
            base = (s * (k + m) + i) * pitch
            flat[base:base + S] = r.integers(0, 256, S, dtype=np.uint8)
    dev = torch.from_numpy(flat).cuda()
    ptrs = [dev.data_ptr() + (s * (k + m) + i) * pitch for s in range(nst) for i in range(k + m)]
    crcs = torch.full((nst * (k + m),), 0x5A5A5A5A, dtype=torch.int32, device="cuda")
    capfd.readouterr()
    rs.New(k, m).encode_crc_batch(ptrs, S, nst, crcs.data_ptr())
    torch.cuda.synchronize()
    assert routed(capfd.readouterr().err, k, m)
    got = dev.cpu().numpy()
    words = crcs.cpu().numpy().view(np.uint32).reshape(nst, k + m)
    host_rows = [[flat[(s * (k + m) + i) * pitch:(s * (k + m) + i) * pitch + S] for i in range(k + m)] for s in range(nst)]
    got_rows = [[got[(s * (k + m) + i) * pitch:(s * (k + m) + i) * pitch + S] for i in range(k + m)] for s in range(nst)]
    check_stripes(k, m, host_rows, got_rows, words)
    # the pad bytes between rows are untouched (tail stores stay inside the row)
    for s in range(nst):
        for i in range(k + m):
            end = (s * (k + m) + i) * pitch + S
            assert not got[end:end + offset].any(), (s, i)


@ec12p4
@pytest.mark.parametrize("S", [17, 2049, 100003])
def test_ec12p4_encode_crc_pointer_table(rs, S, monkeypatch, capfd):
    """Shards in separate allocations: pointer-table launches of 96 / 16 = 6 stripes (13 stripes:
    three launches, the last one short)."""
    monkeypatch.setenv("CFSEC_TRACE_CRC", "1")
    k, m, nst = 12, 4, 13
    r = np.random.default_rng(S)
    sh = [[torch.from_numpy(r.integers(0, 256, S, dtype=np.uint8)).cuda() if i < k
           else torch.zeros(S, dtype=torch.uint8, device="cuda") for i in range(k + m)] for _ in range(nst)]
    host_rows = [[t.cpu().numpy() for t in st] for st in sh]
    ptrs = [t.data_ptr() for st in sh for t in st]
    crcs = torch.zeros(nst * (k + m), dtype=torch.int32, device="cuda")
    capfd.readouterr()
    rs.New(k, m).encode_crc_batch(ptrs, S, nst, crcs.data_ptr())
    torch.cuda.synchronize()
    assert routed(capfd.readouterr().err, k, m)
    words = crcs.cpu().numpy().view(np.uint32).reshape(nst, k + m)
    check_stripes(k, m, host_rows, [[t.cpu().numpy() for t in st] for st in sh], words)


@pytest.mark.parametrize("S", [1, 15, 2047, 2048, 2049, 4097, 65539, 699051])
def test_c4_fused_lrc_encode_crc(S, monkeypatch, capfd):
    """EC6P10L2's fused LRC encode (10 global + 2 local rows over the 6 data shards) with all 18
    checksums through the ec batch seam (what access calls): 7 bids in one allocation at pitch S
    (odd pitches misalign every row), against the ec oracle's Encode and zlib."""
    monkeypatch.setenv("CFSEC_TRACE_CRC", "1")
    from chubaofs_amd import codemode as cm, ec
    from oracle.ec_oracle import ECOracle, Slice
    t = cm.GetTactic(cm.EC6P10L2)
    total, nb = t.N + t.M + t.L, 7
    enc = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=False), device=0)
    orc = ECOracle.from_tactic(t, enable_verify=False)
    r = np.random.default_rng(S + 6)
    data = r.integers(0, 256, (nb, t.N, S), dtype=np.uint8)
    buf = torch.zeros((nb, total, S), dtype=torch.uint8, device="cuda")
    buf[:, :t.N] = torch.from_numpy(data).cuda()
    stripes = [[buf[b, i] for i in range(total)] for b in range(nb)]
    capfd.readouterr()
    st, crcs = enc.EncodeBatch(stripes, crcs=True)
    torch.cuda.synchronize()
    assert routed(capfd.readouterr().err, t.N, t.M + t.L)
    assert st == [0] * nb
    got = buf.cpu().numpy()
    for b in range(nb):
        ref = [Slice.of(data[b, i].copy()) for i in range(t.N)] + [Slice.of(np.zeros(S, np.uint8)) for _ in range(total - t.N)]
        assert orc.encode(ref) == 0
        for i in range(total):
            w = ref[i].view()
            assert np.array_equal(got[b, i], w), (b, i)
            assert crcs[b][i] == crc(w), (b, i, hex(crcs[b][i]), hex(crc(w)))


@ec12p4_long
def test_ec12p4_large_stripe_vs_separate_pass(rs, monkeypatch, capfd):
    """BASELINE C2's shape (S = 5,592,406, 2 stripes): the fused words equal the standalone
    checksum pass over the same shards (cfsec_crc32_ieee_batch), and the parity equals the plain
    encode's."""
    monkeypatch.setenv("CFSEC_TRACE_CRC", "1")
    k, m, S, nst = 12, 4, 5592406, 2
    pitch = (S + 255) // 256 * 256
    g = torch.Generator(device="cuda").manual_seed(0xB5C)
    dev = torch.randint(0, 256, (nst, k + m, pitch), dtype=torch.uint8, device="cuda", generator=g)
    dev[:, k:] = 0
    ptrs = [dev.data_ptr() + (s * (k + m) + i) * pitch for s in range(nst) for i in range(k + m)]
    enc = rs.New(k, m)
    crcs = torch.zeros(nst * (k + m), dtype=torch.int32, device="cuda")
    capfd.readouterr()
    enc.encode_crc_batch(ptrs, S, nst, crcs.data_ptr())
    torch.cuda.synchronize()
    assert routed(capfd.readouterr().err, k, m)
    fused = dev.clone()
    dev[:, k:] = 0
    enc.encode_batch(ptrs, S, nst)
    torch.cuda.synchronize()
    assert torch.equal(dev[:, :, :S], fused[:, :, :S])
    words = crcs.cpu().numpy().view(np.uint32).tolist()
    assert words == rs.crc32_ieee_batch(ptrs, S)


@pytest.mark.skipif(os.environ.get("CFSEC_BS_CRC") is not None, reason="the child process itself")
def test_per_row_form_and_ec12p4_in_child():
    """This module again with CFSEC_BS_CRC=253: every route on, EC12P4's through bit 3."""
    env = dict(os.environ, CFSEC_BS_CRC="253")
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", __file__],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert " passed" in r.stdout and "failed" not in r.stdout, r.stdout[-2000:]


@pytest.mark.parametrize("S", [2049, 65536, 100003])
def test_c4_fused_lrc_encode_crc_scattered(S, monkeypatch, capfd):
    """The same with every shard its own allocation (13 bids: pointer-table launches of 96 / 18 = 5
    bids, the residues of each launch at its own offset of the scratch, one combine)."""
    monkeypatch.setenv("CFSEC_TRACE_CRC", "1")
    from chubaofs_amd import codemode as cm, ec
    from oracle.ec_oracle import ECOracle, Slice
    t = cm.GetTactic(cm.EC6P10L2)
    total, nb = t.N + t.M + t.L, 13
    enc = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=False), device=0)
    orc = ECOracle.from_tactic(t, enable_verify=False)
    r = np.random.default_rng(S + 60)
    data = r.integers(0, 256, (nb, t.N, S), dtype=np.uint8)
    stripes = [[torch.from_numpy(data[b, i].copy()).cuda() if i < t.N else torch.zeros(S, dtype=torch.uint8, device="cuda")
                for i in range(total)] for b in range(nb)]
    capfd.readouterr()
    st, crcs = enc.EncodeBatch(stripes, crcs=True)
    torch.cuda.synchronize()
    assert routed(capfd.readouterr().err, t.N, t.M + t.L)
    assert st == [0] * nb
    for b in range(nb):
        ref = [Slice.of(data[b, i].copy()) for i in range(t.N)] + [Slice.of(np.zeros(S, np.uint8)) for _ in range(total - t.N)]
        assert orc.encode(ref) == 0
        for i in range(total):
            w = ref[i].view()
            assert np.array_equal(stripes[b][i].cpu().numpy(), w), (b, i)
            assert crcs[b][i] == crc(w), (b, i)


@ec16
@pytest.mark.parametrize("S", [1, 2047, 2049, 65539, 262144])
@pytest.mark.parametrize("offset", [0, 5])
def test_ec16p20_encode_crc(rs, S, offset, monkeypatch, capfd):
    """EC16P20's encode + 36 checksums (16 x 20 on the EC16P20L2 network's first 20 rows), 3 stripes
    in one allocation at pitch S + offset."""
    monkeypatch.setenv("CFSEC_TRACE_CRC", "1")
    k, m, nst = 16, 20, 3
    pitch = S + offset
    r = np.random.default_rng(S * 3 + offset)
    flat = np.zeros(nst * (k + m) * pitch + 64, np.uint8)
    for s_ in range(nst):
        for i in range(k):
            base = (s_ * (k + m) + i) * pitch
            flat[base:base + S] = r.integers(0, 256, S, dtype=np.uint8)
    dev = torch.from_numpy(flat).cuda()
    ptrs = [dev.data_ptr() + (s_ * (k + m) + i) * pitch for s_ in range(nst) for i in range(k + m)]
    crcs = torch.full((nst * (k + m),), 0x3C3C3C3C, dtype=torch.int32, device="cuda")
    capfd.readouterr()
    rs.New(k, m).encode_crc_batch(ptrs, S, nst, crcs.data_ptr())
    torch.cuda.synchronize()
    assert routed(capfd.readouterr().err, k, m)
    got = dev.cpu().numpy()
    words = crcs.cpu().numpy().view(np.uint32).reshape(nst, k + m)
    rows = lambda a, s_, i: a[(s_ * (k + m) + i) * pitch:(s_ * (k + m) + i) * pitch + S]
    check_stripes(k, m, [[rows(flat, s_, i) for i in range(k + m)] for s_ in range(nst)],
                  [[rows(got, s_, i) for i in range(k + m)] for s_ in range(nst)], words)


@ec16
@pytest.mark.parametrize("S", [17, 4097, 262144])
def test_ec16p20l2_fused_encode_crc(S, monkeypatch, capfd):
    """EC16P20L2's fused LRC encode (20 global + 2 local rows) with all 38 checksums through the ec
    batch seam, 4 bids in one allocation, against the ec oracle and zlib."""
    monkeypatch.setenv("CFSEC_TRACE_CRC", "1")
    from chubaofs_amd import codemode as cm, ec
    from oracle.ec_oracle import ECOracle, Slice
    t = cm.GetTactic(cm.EC16P20L2)
    total, nb = t.N + t.M + t.L, 4
    enc = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=False), device=0)
    orc = ECOracle.from_tactic(t, enable_verify=False)
    r = np.random.default_rng(S + 16)
    data = r.integers(0, 256, (nb, t.N, S), dtype=np.uint8)
    buf = torch.zeros((nb, total, S), dtype=torch.uint8, device="cuda")
    buf[:, :t.N] = torch.from_numpy(data).cuda()
    stripes = [[buf[b, i] for i in range(total)] for b in range(nb)]
    capfd.readouterr()
    st, crcs = enc.EncodeBatch(stripes, crcs=True)
    torch.cuda.synchronize()
    assert routed(capfd.readouterr().err, t.N, t.M + t.L)
    assert st == [0] * nb
    got = buf.cpu().numpy()
    for b in range(nb):
        ref = [Slice.of(data[b, i].copy()) for i in range(t.N)] + [Slice.of(np.zeros(S, np.uint8)) for _ in range(total - t.N)]
        assert orc.encode(ref) == 0
        for i in range(total):
            w = ref[i].view()
            assert np.array_equal(got[b, i], w), (b, i)
            assert crcs[b][i] == crc(w), (b, i)


RS_MORE = [(6, 8), (6, 10), (12, 9), (15, 12), (10, 4), (4, 4), (3, 3)] if MASK & 16 else []
RS_MORE += [(6, 6), (16, 4)] if MASK & 64 else []
RS_MORE += [(6, 3)] if MASK & 128 else []


@pytest.mark.skipif(not RS_MORE, reason="the other RS modes' routes are off (CFSEC_BS_CRC without bits 4, 6, 7)")
@pytest.mark.parametrize("k,m", RS_MORE or [(0, 0)])
@pytest.mark.parametrize("S", [1, 2049, 65539])
def test_other_rs_modes_encode_crc(rs, k, m, S, monkeypatch, capfd):
    """EC6P8 / EC6P10 / EC6P6 / EC6P3 (the EC6P10L2 network's first rows), EC16P4 (the 16 + 20
    network's), EC12P9, EC15P12 and EC3P3 (unpaired: k odd), EC10P4 and EC4P4 encodes with every
    shard checksummed, 3 stripes at an odd pitch."""
    monkeypatch.setenv("CFSEC_TRACE_CRC", "1")
    nst, pitch = 3, S + 3
    r = np.random.default_rng(k * 1000 + m * 10 + S)
    flat = np.zeros(nst * (k + m) * pitch + 64, np.uint8)
    for s_ in range(nst):
        for i in range(k):
            base = (s_ * (k + m) + i) * pitch
            flat[base:base + S] = r.integers(0, 256, S, dtype=np.uint8)
    dev = torch.from_numpy(flat).cuda()
    ptrs = [dev.data_ptr() + (s_ * (k + m) + i) * pitch for s_ in range(nst) for i in range(k + m)]
    crcs = torch.full((nst * (k + m),), 0x77, dtype=torch.int32, device="cuda")
    capfd.readouterr()
    rs.New(k, m).encode_crc_batch(ptrs, S, nst, crcs.data_ptr())
    torch.cuda.synchronize()
    assert routed(capfd.readouterr().err, k, m)
    got = dev.cpu().numpy()
    words = crcs.cpu().numpy().view(np.uint32).reshape(nst, k + m)
    rows = lambda a, s_, i: a[(s_ * (k + m) + i) * pitch:(s_ * (k + m) + i) * pitch + S]
    check_stripes(k, m, [[rows(flat, s_, i) for i in range(k + m)] for s_ in range(nst)],
                  [[rows(got, s_, i) for i in range(k + m)] for s_ in range(nst)], words)


@rs_more
@pytest.mark.parametrize("mode", ["EC6P3L3", "EC4P4L2", "EC6P6L9", "EC6P8L10"])
@pytest.mark.parametrize("S", [17, 2049, 65539])
def test_other_lrc_fused_encode_crc(mode, S, monkeypatch, capfd):
    """The other LRC modes' fused encodes (global + every AZ's local rows over the data, as
    lrcencoder.go's Encode fills them) with every shard checksummed, through the ec batch seam: 3 bids
    in one allocation, against the ec oracle's Encode and zlib."""
    monkeypatch.setenv("CFSEC_TRACE_CRC", "1")
    from chubaofs_amd import codemode as cm, ec
    from oracle.ec_oracle import ECOracle, Slice
    t = cm.GetTactic(getattr(cm, mode))
    total, nb = t.N + t.M + t.L, 3
    enc = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=False), device=0)
    orc = ECOracle.from_tactic(t, enable_verify=False)
    r = np.random.default_rng(S + total)
    data = r.integers(0, 256, (nb, t.N, S), dtype=np.uint8)
    buf = torch.zeros((nb, total, S), dtype=torch.uint8, device="cuda")
    buf[:, :t.N] = torch.from_numpy(data).cuda()
    stripes = [[buf[b, i] for i in range(total)] for b in range(nb)]
    capfd.readouterr()
    st, crcs = enc.EncodeBatch(stripes, crcs=True)
    torch.cuda.synchronize()
    assert routed(capfd.readouterr().err, t.N, t.M + t.L), mode
    assert st == [0] * nb
    got = buf.cpu().numpy()
    for b in range(nb):
        ref = [Slice.of(data[b, i].copy()) for i in range(t.N)] + [Slice.of(np.zeros(S, np.uint8)) for _ in range(total - t.N)]
        assert orc.encode(ref) == 0
        for i in range(total):
            w = ref[i].view()
            assert np.array_equal(got[b, i], w), (mode, b, i)
            assert crcs[b][i] == crc(w), (mode, b, i)


@plain
@pytest.mark.parametrize("mode", ["EC6P6L9", "EC6P8L10"])
@pytest.mark.parametrize("S", [17, 2049, 65539])
def test_wide_lrc_plain_encode(mode, S, monkeypatch, capfd):
    """EC6P6L9's / EC6P8L10's fused encode without checksums on the bit-sliced product (one pass over
    the inputs instead of two fixed-K products), 3 bids, against the ec oracle's Encode."""
    monkeypatch.setenv("CFSEC_TRACE_CRC", "1")
    from chubaofs_amd import codemode as cm, ec
    from oracle.ec_oracle import ECOracle, Slice
    t = cm.GetTactic(getattr(cm, mode))
    total, nb = t.N + t.M + t.L, 3
    enc = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=False), device=0)
    orc = ECOracle.from_tactic(t, enable_verify=False)
    r = np.random.default_rng(S + 3 * total)
    data = r.integers(0, 256, (nb, t.N, S), dtype=np.uint8)
    buf = torch.zeros((nb, total, S), dtype=torch.uint8, device="cuda")
    buf[:, :t.N] = torch.from_numpy(data).cuda()
    stripes = [[buf[b, i] for i in range(total)] for b in range(nb)]
    capfd.readouterr()
    st = enc.EncodeBatch(stripes)
    torch.cuda.synchronize()
    assert f"bs plain k={t.N} m={t.M + t.L}" in capfd.readouterr().err, mode
    assert list(st) == [0] * nb
    got = buf.cpu().numpy()
    for b in range(nb):
        ref = [Slice.of(data[b, i].copy()) for i in range(t.N)] + [Slice.of(np.zeros(S, np.uint8)) for _ in range(total - t.N)]
        assert orc.encode(ref) == 0
        for i in range(total):
            assert np.array_equal(got[b, i], ref[i].view()), (mode, b, i)
