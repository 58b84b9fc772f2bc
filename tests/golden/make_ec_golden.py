"""Generates tests/golden/ec_golden.json -- TEST INFRASTRUCTURE.

Golden vectors for the coding path, computed with the CPU oracle (oracle/gf_oracle.c, the
klauspost/reedsolomon v1.11.7 restatement pinned by tests/test_oracle.py) and the code-mode
layout of chubaofs_amd/codemode.py (pinned by tests/test_codemode.py), as SURVEY §8(c) lists:

  * the systematic matrices buildMatrix(k, k+m) of the code-mode shapes (KRS/reedsolomon.go:220-244);
  * decode matrices (inverse of the first k surviving rows) for selected erasure sets;
  * blobnode's mock stripes (blobnode/worker_for_test.go:62-69, 79-83, 103-140): bids 1..7 with
    shard sizes {1024, 2048, 0, 512, 23, 65, 12}, data shard i of bid b = genMockBytes(b + i, size),
    global parity by Reconstruct, then every AZ-local parity -- recorded as SHA-256 and
    crc32.ChecksumIEEE of every shard, plus the full parity bytes of the smallest sizes.

Run from the repo root:  python tests/golden/make_ec_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from chubaofs_amd import codemode as cm  # noqa: E402
from oracle import oracle as O  # noqa: E402

SHAPES = [(6, 6), (12, 4), (6, 10), (8, 1), (16, 20), (18, 1)]
ERASURES = {"12,4": [[0, 1, 2, 3], [3, 13], [12, 13, 14, 15]], "6,6": [[0, 5, 6, 11], [1]],
            "16,20": [[0, 1, 16, 17], list(range(20))], "6,10": [[2, 9], [0, 1, 2, 3, 4, 5]]}
MODES = [cm.EC6P6, cm.EC12P4, cm.EC6P10L2, cm.EC16P20L2]
BIDS = [1, 2, 3, 4, 5, 6, 7]
SIZES = [1024, 2048, 0, 512, 23, 65, 12]
FULL_BYTES_MAX = 65  # parity bytes kept verbatim up to this shard size


def gen_mock_bytes(letter: int, size: int) -> np.ndarray:
    """blobnode/worker_for_test.go:62-69."""
    return ((letter + np.arange(size)) & 0xFF).astype(np.uint8)


def mock_stripe(mode: int, bid: int, size: int):
    """All N+M+L shards of one mock bid (worker_for_test.go:103-140)."""
    t = cm.GetTactic(mode)
    glob, n, m = t.GlobalStripe()
    shards = [None] * (t.N + t.M + t.L)
    for i in glob[:n]:
        shards[i] = gen_mock_bytes(bid + i, size)
    for i in glob[n:n + m]:
        shards[i] = np.zeros(size, np.uint8)
    g = [shards[i] for i in glob]
    assert O.encode(n, m, g) == 0
    for i, s in zip(glob, g):
        shards[i] = s
    if t.L:
        locals_, ln, lm = t.AllLocalStripe()
        for stripe in locals_:
            for i in stripe[ln:ln + lm]:
                shards[i] = np.zeros(size, np.uint8)
            ls = [shards[i] for i in stripe]
            assert O.encode(ln, lm, ls) == 0
    return shards


def decode_matrix(k: int, m: int, erased):
    full = O.build_matrix(k, k + m)
    survivors = [i for i in range(k + m) if i not in erased][:k]
    err, inv = O.invert(full[survivors])
    assert err == 0
    return survivors, inv


def main():
    out = {"generator": "tests/golden/make_ec_golden.py (CPU oracle)", "matrices": {}, "decode": {}, "stripes": {}}
    for k, m in SHAPES:
        out["matrices"][f"{k},{m}"] = O.build_matrix(k, k + m).tobytes().hex()
    for key, sets in ERASURES.items():
        k, m = map(int, key.split(","))
        for erased in sets:
            survivors, inv = decode_matrix(k, m, erased)
            out["decode"][f"{key}:{','.join(map(str, erased))}"] = {"survivors": survivors, "inverse": inv.tobytes().hex()}
    for mode in MODES:
        rows = []
        for bid, size in zip(BIDS, SIZES):
            if size == 0:
                rows.append({"bid": bid, "size": 0})
                continue
            shards = mock_stripe(mode, bid, size)
            row = {"bid": bid, "size": size,
                   "sha256": [hashlib.sha256(s.tobytes()).hexdigest()[:32] for s in shards],
                   "crc32": [O.crc32_ieee(s) for s in shards]}
            if size <= FULL_BYTES_MAX:
                t = cm.GetTactic(mode)
                row["parity_hex"] = [shards[i].tobytes().hex() for i in range(t.N, t.N + t.M + t.L)]
            rows.append(row)
        out["stripes"][cm.Name(mode)] = rows
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ec_golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(f"wrote {path} ({os.path.getsize(path)} bytes)")


if __name__ == "__main__":
    main()
