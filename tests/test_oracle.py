"""The oracle itself: pinned against the reference's own data, checked against an
independent pure-Python restatement, and exercised on the reference's round-trip
invariants.  CPU only."""
import hashlib
import itertools
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_tables_match_reference_literals():
    """KRS/galois.go:28-937 literal tables, via tests/golden/tables.json (SHA-256 of the
    reference text's values, made by tests/golden/make_table_fixture.py)."""
    fx = json.load(open(os.path.join(GOLDEN, "tables.json")))["tables"]
    t = O.tables()
    assert set(fx) == set(t)
    for name, arr in t.items():
        w = fx[name]["width"]
        blob = arr.astype("<u8").tobytes() if w == 8 else arr.astype(np.uint8).tobytes()
        assert arr.size == fx[name]["count"], name
        assert hashlib.sha256(blob).hexdigest() == fx[name]["sha256"], name


# ---- an independent pure-Python restatement (KRS/galois.go, KRS/matrix.go) ----
def _py_field():
    exp = [0] * 510
    log = [0] * 256
    x = 1
    for i in range(255):
        exp[i] = exp[i + 255] = x
        log[x] = i
        x <<= 1
        if x & 0x100:
            x ^= 0x11D
    return exp, log


EXP, LOG = _py_field()


def py_mul(a, b):
    return 0 if a == 0 or b == 0 else EXP[LOG[a] + LOG[b]]


def py_div(a, b):
    return 0 if a == 0 else EXP[(LOG[a] - LOG[b]) % 255]


def py_exp(a, n):
    if n == 0:
        return 1
    if a == 0:
        return 0
    return EXP[(LOG[a] * n) % 255]


def py_invert(m):
    n = len(m)
    w = [list(r) + [1 if i == j else 0 for j in range(n)] for i, r in enumerate(m)]
    for r in range(n):
        if w[r][r] == 0:
            for b in range(r + 1, n):
                if w[b][r]:
                    w[r], w[b] = w[b], w[r]
                    break
        if w[r][r] == 0:
            raise ZeroDivisionError("singular")
        s = py_div(1, w[r][r])
        w[r] = [py_mul(v, s) for v in w[r]]
        for b in range(n):
            if b != r and w[b][r]:
                s = w[b][r]
                w[b] = [v ^ py_mul(s, u) for v, u in zip(w[b], w[r])]
    return [row[n:] for row in w]


def py_build(k, total):
    vm = [[py_exp(r, c) for c in range(k)] for r in range(total)]
    inv = py_invert(vm[:k])
    out = []
    for r in range(total):
        row = []
        for c in range(k):
            v = 0
            for i in range(k):
                v ^= py_mul(vm[r][i], inv[i][c])
            row.append(v)
        out.append(row)
    return out


@pytest.mark.parametrize("k,m", [(6, 6), (12, 4), (6, 10), (8, 1), (16, 20), (18, 1), (15, 12), (3, 3),
                                 (16, 4), (10, 4), (6, 3), (12, 9), (4, 4), (6, 8)])
def test_build_matrix_two_restatements_agree(k, m):
    c = O.build_matrix(k, k + m)
    p = np.array(py_build(k, k + m), np.uint8)
    assert np.array_equal(c, p)
    assert np.array_equal(c[:k], np.eye(k, dtype=np.uint8))  # systematic


def test_survey_checkpoints():
    """SURVEY.md appendix A values (a separate transcription made during the survey)."""
    h = lambda row: " ".join("%02x" % v for v in row)
    m = O.build_matrix(12, 16)
    assert h(m[12]) == "af b4 96 8c f5 e8 c4 d8 1b 1c 12 14"
    assert h(m[13]) == "b4 af 8c 96 e8 f5 d8 c4 1c 1b 14 12"
    assert h(m[14]) == "96 8c af b4 c4 d8 f5 e8 12 14 1b 1c"
    assert h(m[15]) == "8c 96 b4 af d8 c4 e8 f5 14 12 1c 1b"
    m6 = O.build_matrix(6, 12)
    assert [h(m6[6 + i]) for i in range(4)] == ["07 06 05 04 03 02", "06 07 04 05 02 03",
                                                "a0 df df b7 fe e8", "df a0 b7 df e8 fe"]
    assert np.array_equal(O.build_matrix(6, 16)[6:10], m6[6:10])
    assert h(O.build_matrix(8, 9)[8]) == "1a 84 ba 33 e7 10 c6 27"
    assert h(O.build_matrix(18, 19)[18]) == "e2 05 31 d6 cf 22 08 e5 af a2 b5 b8 42 44 4e 48 03 02"
    assert h(O.build_matrix(16, 36)[16]) == "21 b5 f6 85 df 02 b7 87 3e dd 4a a4 8d da 61 30"
    sh = [np.array([i + 1], np.uint8) for i in range(12)] + [np.zeros(1, np.uint8) for _ in range(4)]
    assert O.encode(12, 4, sh) == 0
    assert [int(s[0]) for s in sh[12:]] == [0x9E, 0x7D, 0x01, 0xEE]
    err, dec = O.invert(m[4:16])
    assert err == 0
    assert h(dec[0]) == "1b 1c 12 14 f5 e8 c4 d8 af b4 96 8c"
    assert h(dec[3]) == "14 12 1c 1b d8 c4 e8 f5 8c 96 b4 af"
    assert O.crc32_ieee(b"123456789") == 0xCBF43926


def test_gal_exp_semantics():
    assert O.lib().oracle_gal_exp(0, 0) == 1  # galExp(0,0) == 1 (KRS/galois.go:892-897)
    assert O.lib().oracle_gal_exp(0, 3) == 0
    for a in (1, 2, 3, 29, 255):
        for n in range(0, 300, 37):
            assert O.lib().oracle_gal_exp(a, n) == py_exp(a, n)


def test_mul_table_is_the_field():
    t = O.tables()["mulTable"]
    for a in range(0, 256, 7):
        for b in range(0, 256, 11):
            assert t[a, b] == py_mul(a, b)


def test_singular_detected():
    err, _ = O.invert(np.array([[1, 2], [2, 4]], np.uint8))  # row 2 = 2*row 1
    assert err == 8


def gen_mock_bytes(letter, size):
    """blobnode/worker_for_test.go:62-69"""
    return np.array([(letter + i) & 0xFF for i in range(size)], np.uint8)


@pytest.mark.parametrize("k,m", [(6, 6), (12, 4), (6, 10), (16, 20), (15, 12), (4, 4)])
def test_oracle_round_trips_mock_bids(k, m):
    """worker_for_test.go bid sizes {1024,2048,0,512,23,65,12}: encode, drop up to m shards,
    reconstruct, verify (the blobnode repair loop, work_shard_recover.go:708-771)."""
    for size in (1024, 2048, 512, 23, 65, 12):
        sh = [gen_mock_bytes(ord("A") + i, size) for i in range(k)] + [np.zeros(size, np.uint8) for _ in range(m)]
        assert O.encode(k, m, sh) == 0
        assert O.verify(k, m, sh) == (0, True)
        for erased in [tuple(range(m)), tuple(range(k + m - m, k + m)), tuple(range(0, k + m, 2))[:m]]:
            work = [s.copy() for s in sh]
            for i in erased:
                work[i][:] = 0
            err, filled = O.reconstruct(k, m, work, [i not in erased for i in range(k + m)])
            assert err == 0
            for i in range(k + m):
                assert np.array_equal(work[i], sh[i])
    # zero-size bid: checkShards -> ErrShardNoData
    z = [np.zeros(0, np.uint8) for _ in range(k + m)]
    assert O.encode(k, m, z) == 2


def test_oracle_reconstruct_selection_rules():
    k, m, size = 12, 4, 40
    r = np.random.default_rng(1)
    sh = [r.integers(0, 256, size, dtype=np.uint8) for _ in range(k)] + [np.zeros(size, np.uint8) for _ in range(m)]
    O.encode(k, m, sh)
    # too few
    err, _ = O.reconstruct(k, m, [s.copy() for s in sh], [i >= 5 for i in range(16)])
    assert err == 1
    # data-only with all data present: nothing filled
    err, filled = O.reconstruct(k, m, [s.copy() for s in sh], [i < 12 for i in range(16)], data_only=True)
    assert err == 0 and not any(filled)
    # data-only leaves missing parity unfilled
    err, filled = O.reconstruct(k, m, [s.copy() for s in sh], [i not in (0, 13) for i in range(16)], True)
    assert err == 0 and filled[0] and not filled[13]
    # size mismatch among present shards
    bad = [s.copy() for s in sh]
    bad[3] = bad[3][:10]
    assert O.encode(k, m, bad) == 3


def test_simd_baseline_matches_oracle():
    feats = O.simd_features()
    if not feats["avx2"]:
        pytest.skip("no AVX2 on this host")
    for k, m in [(12, 4), (6, 6), (16, 20), (8, 1), (10, 10)]:
        rows = O.build_matrix(k, k + m)[k:]
        for S in (1, 63, 64, 65, 4097, 100003):
            r = np.random.default_rng(S + k)
            ins = [r.integers(0, 256, S, dtype=np.uint8) for _ in range(k)]
            want = ins + [np.zeros(S, np.uint8) for _ in range(m)]
            O.encode(k, m, want)
            modes = [1] + ([2] if feats["gfni"] and k <= 10 and m <= 10 else [])
            for force in modes:
                for threads in (1, 3):
                    outs = [np.zeros(S, np.uint8) for _ in range(m)]
                    O.simd_code(rows, ins, outs, threads, force)
                    for i in range(m):
                        assert np.array_equal(outs[i], want[k + i]), (k, m, S, force, threads)


def test_crc32_incremental():
    r = np.random.default_rng(3)
    b = r.integers(0, 256, 10000, dtype=np.uint8)
    import zlib
    assert O.crc32_ieee(b) == zlib.crc32(b.tobytes())
    assert O.lib().oracle_crc32_update(O.crc32_ieee(b[:4000]), b[4000:].ctypes.data, 6000) == zlib.crc32(b.tobytes())
