"""Where the lookup-product kernel's clamped row end goes wrong (dev probe, round 5): EC12P9-shaped
products through the reedsolomon API at a few sizes, every row against the oracle, the first
mismatching byte and the count per row.  CFSEC_LIB_PATH picks the library under test."""
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from chubaofs_amd import reedsolomon  # noqa: E402
from oracle import oracle as O  # noqa: E402


def dev(a):
    return [torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in a]


def host(ts):
    torch.cuda.synchronize()
    return [t.cpu().numpy() for t in ts]


def report(tag, got, want, rows):
    bad = []
    for i in rows:
        d = np.nonzero(got[i] != want[i])[0]
        if len(d):
            bad.append((i, len(d), int(d[0]), int(d[-1])))
    print(f"{tag}: {'OK' if not bad else bad}", flush=True)


for k, m in ((12, 9), (15, 12), (16, 8)):
    enc = reedsolomon.New(k, m)
    for S in (512, 513, 100, 4096, 4100):
        r = np.random.default_rng(S + k)
        sh = [r.integers(0, 256, S, dtype=np.uint8) for _ in range(k)] + [np.zeros(S, np.uint8) for _ in range(m)]
        assert O.encode(k, m, sh) == 0
        d = dev([s if i < k else np.zeros(S, np.uint8) for i, s in enumerate(sh)])
        enc.Encode(d)
        report(f"({k},{m}) S={S} encode", host(d), sh, range(k, k + m))
        print(f"   verify of the golden: {enc.Verify(dev(sh))}", flush=True)
        rnd = random.Random(S)
        for trial in range(3):
            erased = sorted(rnd.sample(range(k + m), m))
            dd = dev([s if i not in erased else s[:0] for i, s in enumerate(sh)])
            try:
                enc.Reconstruct(dd)
                report(f"   reconstruct {erased}", host(dd), sh, range(k + m))
            except Exception as e:  # noqa: BLE001
                print(f"   reconstruct {erased}: {e}")
