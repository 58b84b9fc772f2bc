"""Golden EC vectors (tests/golden/ec_golden.json, made by tests/golden/make_ec_golden.py): the
oracle must keep reproducing them (CPU), and the GPU engine must produce the same bytes (gpu).

The vectors are SURVEY §8(c)'s list: the systematic matrices of the code-mode shapes, decode
matrices for selected erasure sets, and blobnode's mock stripes (blobnode/worker_for_test.go:
62-140; bids 1..7, sizes {1024, 2048, 0, 512, 23, 65, 12}) with global and AZ-local parity.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from chubaofs_amd import codemode as cm
from oracle import oracle as O

GOLDEN = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "ec_golden.json")))
MODES = {cm.Name(m): m for m in (cm.EC6P6, cm.EC12P4, cm.EC6P10L2, cm.EC16P20L2)}


def gen_mock_bytes(letter, size):
    return ((letter + np.arange(size)) & 0xFF).astype(np.uint8)


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()[:32]


def data_shards(mode, bid, size):
    """Data shards of a mock bid; parity / local slots zero-filled."""
    t = cm.GetTactic(mode)
    glob, n, _ = t.GlobalStripe()
    shards = [np.zeros(size, np.uint8) for _ in range(t.N + t.M + t.L)]
    for i in glob[:n]:
        shards[i] = gen_mock_bytes(bid + i, size)
    return shards


def test_matrices_reproduce():
    for key, hx in GOLDEN["matrices"].items():
        k, m = map(int, key.split(","))
        assert O.build_matrix(k, k + m).tobytes().hex() == hx, key
    # EC12P4 parity row 0
    assert GOLDEN["matrices"]["12,4"][2 * 144:2 * 156] == "afb4968cf5e8c4d81b1c1214"


def test_decode_matrices_reproduce():
    for key, v in GOLDEN["decode"].items():
        shape, erased = key.split(":")
        k, m = map(int, shape.split(","))
        erased = [int(x) for x in erased.split(",")]
        full = O.build_matrix(k, k + m)
        survivors = [i for i in range(k + m) if i not in erased][:k]
        assert survivors == v["survivors"]
        err, inv = O.invert(full[survivors])
        assert err == 0 and inv.tobytes().hex() == v["inverse"], key
        # and it is the inverse
        prod = np.zeros((k, k), np.uint8)
        for r in range(k):
            for c in range(k):
                acc = 0
                for j in range(k):
                    acc ^= O.gal_mul(int(inv[r, j]), int(full[survivors][j, c]))
                prod[r, c] = acc
        assert np.array_equal(prod, np.eye(k, dtype=np.uint8)), key


@pytest.mark.parametrize("name", sorted(MODES))
def test_mock_stripes_reproduce_on_oracle(name):
    mode = MODES[name]
    t = cm.GetTactic(mode)
    for row in GOLDEN["stripes"][name]:
        if row["size"] == 0:
            continue
        shards = data_shards(mode, row["bid"], row["size"])
        glob, n, m = t.GlobalStripe()
        g = [shards[i] for i in glob]
        assert O.encode(n, m, g) == 0
        if t.L:
            locals_, ln, lm = t.AllLocalStripe()
            for stripe in locals_:
                ls = [shards[i] for i in stripe]
                assert O.encode(ln, lm, ls) == 0
        assert [digest(s) for s in shards] == row["sha256"], (name, row["bid"])
        assert [O.crc32_ieee(s) for s in shards] == row["crc32"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(MODES))
@pytest.mark.parametrize("memory", ["host", "device"])
def test_mock_stripes_on_gpu(name, memory):
    """ec.Encoder.Encode on the GPU gives the golden bytes of every shard (global + local parity),
    and rebuilding the first M shards gives them back."""
    torch = pytest.importorskip("torch")
    from chubaofs_amd import ec
    mode = MODES[name]
    t = cm.GetTactic(mode)
    enc = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=True))
    for row in GOLDEN["stripes"][name]:
        if row["size"] == 0:
            continue
        shards = data_shards(mode, row["bid"], row["size"])
        if memory == "device":
            shards = [torch.from_numpy(s).cuda() for s in shards]
        enc.Encode(shards)
        got = [s.cpu().numpy() if memory == "device" else s for s in shards]
        assert [digest(s) for s in got] == row["sha256"], (name, row["bid"])
        if "parity_hex" in row:
            assert [s.tobytes().hex() for s in got[t.N:]] == row["parity_hex"]
        bad = list(range(t.M))
        for i in bad:
            shards[i] = shards[i][:0]
        enc.Reconstruct(shards, bad)
        got = [s.cpu().numpy() if memory == "device" else s for s in shards]
        assert [digest(s) for s in got] == row["sha256"], (name, row["bid"], "reconstruct")
