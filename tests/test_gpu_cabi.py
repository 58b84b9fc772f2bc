"""The deployment boundary without PyTorch: tests/cabi/cabi_driver (plain C, built by build()) links
libcfsec.so and drives it the way the cgo shim does -- host shard vectors (pageable and
cfsec_host_alloc), reedsolomon.Encoder and ec.Encoder calls, the blobnode repair batch, crc32block
framing, and the error codes the shim maps to Go sentinels.  The child process never loads torch,
so the library runs on /opt/rocm's HIP runtime (what a Go/C process gets); every record it writes
is checked here against the oracle.
"""
import os
import struct
import subprocess
import zlib

import numpy as np
import pytest

from chubaofs_amd import _lib
from oracle import oracle as O

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "tests", "cabi", "cabi_driver")


def records(path):
    out = {}
    with open(path, "rb") as f:
        data = f.read()
    pos = 0
    while pos < len(data):
        name = data[pos:pos + 16].rstrip(b"\0").decode()
        (n,) = struct.unpack("<Q", data[pos + 16:pos + 24])
        out.setdefault(name, []).append(np.frombuffer(data[pos + 24:pos + 24 + n], np.uint8).copy())
        pos += 24 + n
    return out


def as_int(a):
    return int(np.frombuffer(a.tobytes(), np.int32)[0])


@pytest.fixture(scope="module")
def run(tmp_path_factory):
    assert os.path.exists(DRIVER), "build() compiles tests/cabi/cabi_driver"
    out = tmp_path_factory.mktemp("cabi") / "out.bin"
    env = {k: v for k, v in os.environ.items() if not k.startswith("PYTHON")}
    r = subprocess.run([DRIVER, str(out)], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return records(out)


def split(buf, n):
    return [x.copy() for x in np.split(buf, n)]


def test_runtime_is_opt_rocm(run):
    path = run["hip_runtime"][0].tobytes().decode()
    assert "libamdhip64" in path and "torch" not in path, path
    assert as_int(run["devices"][0]) >= 1


def test_reedsolomon_seam(run):
    k, m = 12, 4
    page = split(run["enc_page"][0], 16)
    want = [x.copy() for x in page[:k]] + [np.zeros_like(page[0]) for _ in range(m)]
    assert O.encode(k, m, want) == 0
    for i in range(16):
        assert np.array_equal(page[i], want[i]), i
    assert as_int(run["verify_ok"][0]) == 1 and as_int(run["verify_bad"][0]) == 0
    assert np.array_equal(run["enc_pin"][0], run["enc_page"][0])
    crcs = np.frombuffer(run["enc_crc"][0].tobytes(), np.uint32)
    assert [int(c) for c in crcs] == [zlib.crc32(x.tobytes()) & 0xFFFFFFFF for x in want]
    assert np.array_equal(run["rec_page"][0], run["enc_page"][0]) and as_int(run["rec_lens"][0]) == 1


def test_error_codes(run):
    assert as_int(run["err_size"][0]) == _lib.ErrShardSize.status
    assert as_int(run["err_few"][0]) == _lib.ErrTooFewShards.status
    assert as_int(run["err_num"][0]) == _lib.ErrTooFewShards.status
    assert as_int(run["err_new"][0]) == _lib.ErrInvShardNum.status
    assert as_int(run["err_max"][0]) == _lib.ErrNotSupported.status


def test_lrc_encoder(run):
    from chubaofs_amd import codemode as cm
    t = cm.GetTactic(cm.EC6P10L2)
    sh = split(run["lrc_enc"][0], t.N + t.M + t.L)
    want = [x.copy() for x in sh[:t.N]] + [np.zeros_like(sh[0]) for _ in range(t.M + t.L)]
    assert O.encode(t.N, t.M, want[:t.N + t.M]) == 0
    ln, lm = (t.N + t.M) // t.AZCount, t.L // t.AZCount
    for az in range(t.AZCount):
        idx, _, _ = t.LocalStripeInAZ(az)
        local = [want[i] for i in idx]
        assert O.encode(ln, lm, local) == 0
    for i in range(len(sh)):
        assert np.array_equal(sh[i], want[i]), i
    assert as_int(run["lrc_ok"][0]) == 1


def test_repair_batch(run):
    k, m = 12, 4
    bads = [[1, 2, 3, 4], [0, 15], [7, 9, 12]]
    status = list(np.frombuffer(run["batch_status"][0].tobytes(), np.int32))
    for b in range(3):
        good = split(run["batch_good"][b], 16)
        src = [x.copy() for x in good]
        assert O.encode(k, m, [x.copy() for x in good[:k]] + [np.zeros_like(good[0])] * m) == 0
        for i in bads[b]:
            src[i][:] = 0
        if b == 2:
            src[14][100] ^= 0x40
        present = [i not in bads[b] for i in range(16)]
        err, _ = O.reconstruct(k, m, src, present)
        assert err == 0
        err, ok = O.verify(k, m, src)
        assert err == 0
        want_status = 0 if ok else _lib.ErrVerify.status
        assert status[b] == want_status, (b, status)
        after = split(run["batch_after"][b], 16)
        for i in range(16):
            assert np.array_equal(after[i], src[i]), (b, i)
    assert status == [0, 0, _lib.ErrVerify.status]


def test_crc32block(run):
    payload = run["blk_payload"][0]
    assert np.array_equal(run["blk_framed"][0], O.crc32block_encode(payload))
    assert int(np.frombuffer(run["blk_crc"][0].tobytes(), np.uint32)[0]) == zlib.crc32(payload.tobytes()) & 0xFFFFFFFF
    assert np.array_equal(run["blk_back"][0], payload[1000:])
    assert as_int(run["blk_mismatch"][0]) == _lib.ErrMismatchedCrc.status
    assert as_int(run["blk_badblock"][0]) == 1
    assert as_int(run["blk_short"][0]) == _lib.ErrShortData.status


def test_contiguous_stripes(run):
    """cfsec_*_contig (ec.Buffer's one-allocation layout, the Go 1.17 cgo path): encode, verify,
    reconstruct of data/global/local shards, the reedsolomon seam with missing shards, the encode
    batch and the repair tasklet with checksums -- against the ec oracle and zlib."""
    from chubaofs_amd import codemode as cm
    from oracle.ec_oracle import ECOracle, Slice
    t = cm.GetTactic(cm.EC6P10L2)
    LT = t.N + t.M + t.L
    CS, CST = 4097, 4100
    enc = run["ct_enc"][0].reshape(LT, CST)
    want = [Slice.of(enc[i, :CS]) for i in range(t.N)] + [Slice(np.zeros(CS, np.uint8)) for _ in range(t.M + t.L)]
    orc = ECOracle.from_tactic(t, enable_verify=True)
    assert orc.encode(want) == 0
    for i in range(LT):
        assert np.array_equal(enc[i, :CS], want[i].view()), i
        assert not enc[i, CS:].any(), i  # the gaps between shards are not touched
    assert as_int(run["ct_ok"][0]) == 1
    rec = run["ct_rec"][0].reshape(LT, CST)
    for i in range(LT):
        assert np.array_equal(rec[i, :CS], want[i].view()), i
    rs_enc = split(run["ct_rs_enc"][0], 16)
    ref = [x.copy() for x in rs_enc[:12]] + [np.zeros(5000, np.uint8) for _ in range(4)]
    assert O.encode(12, 4, ref) == 0
    assert all(np.array_equal(a, b) for a, b in zip(rs_enc, ref))
    assert all(np.array_equal(a, b) for a, b in zip(split(run["ct_rs_rec"][0], 16), ref))
    # encode batch with checksums
    batch = run["ct_batch"][0].reshape(3, LT, 3000)
    crc = np.frombuffer(run["ct_batch_crc"][0].tobytes(), np.uint32).reshape(3, LT)
    assert list(np.frombuffer(run["ct_batch_st"][0].tobytes(), np.int32)) == [0, 0, 0]
    for s in range(3):
        w = [Slice.of(batch[s, i]) for i in range(t.N)] + [Slice(np.zeros(3000, np.uint8)) for _ in range(t.M + t.L)]
        assert orc.encode(w) == 0
        for i in range(LT):
            assert np.array_equal(batch[s, i], w[i].view()), (s, i)
            assert int(crc[s, i]) == zlib.crc32(w[i].view().tobytes()) & 0xFFFFFFFF, (s, i)
    # repair tasklet: bid 0 (3000 B, bad {0, 16}) and bid 1 (1500 B, bad {5, 17})
    good = run["ct_tasklet_good"][0]
    after = run["ct_tasklet"][0]
    assert np.array_equal(after, good)
    off1 = LT * 3000 + 64
    crc = np.frombuffer(run["ct_tasklet_crc"][0].tobytes(), np.uint32).reshape(2, LT)
    assert list(np.frombuffer(run["ct_tasklet_st"][0].tobytes(), np.int32)) == [0, 0]
    for b, (o, S, bad) in enumerate([(0, 3000, [0, 16]), (off1, 1500, [5, 17])]):
        for i in range(LT):
            shard = good[o + i * S:o + (i + 1) * S]
            assert int(crc[b, i]) == ((zlib.crc32(shard.tobytes()) & 0xFFFFFFFF) if i in bad else 0), (b, i)
    assert as_int(run["ct_err_overlap"][0]) == _lib.ErrInvalidArg.status


def test_tasklet_of_separate_pinned_shards(run):
    """blobnode's tasklet with every shard its own cfsec_host_alloc block (the ShardsBuf layout the
    Go 1.17 shim passes without copies): cfsec_ec_reconstruct_batch_crc over EC6P10L2 bids with bad
    {0, 7, 16} and {3, 17}, bid 1 with a corrupted surviving global parity -- statuses, rebuilt bytes
    and checksums against the ec oracle and zlib."""
    from chubaofs_amd import codemode as cm
    from oracle.ec_oracle import ECOracle, Slice
    t = cm.GetTactic(cm.EC6P10L2)
    LT = t.N + t.M + t.L
    good = run["pv_good"]
    after = run["pv_after"]
    st = list(np.frombuffer(run["pv_st"][0].tobytes(), np.int32))
    crc = np.frombuffer(run["pv_crc"][0].tobytes(), np.uint32).reshape(2, LT)
    orc = ECOracle.from_tactic(t)
    for b, bad in enumerate([[0, 7, 16], [3, 17]]):
        sh = [Slice.of(good[b * LT + i]) for i in range(LT)]
        for i in bad:
            sh[i].buf[:] = 0x3C
        if b == 1:
            sh[9].buf[11] ^= 0x80
        want = orc.repair(sh, bad)
        assert st[b] == want, (b, st)
        for i in range(LT):
            assert np.array_equal(after[b * LT + i], sh[i].view()), (b, i)
            if want == 0:
                assert int(crc[b, i]) == ((zlib.crc32(sh[i].view().tobytes()) & 0xFFFFFFFF) if i in bad else 0), (b, i)
    assert st == [0, _lib.ErrVerify.status]
