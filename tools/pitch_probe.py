"""Dev tool: does the HBM placement of the shard rows change the EC12P4 kernel's rate?

Times encode (E) and alternating encode/reconstruct (A) over the bench's 8 x EC12P4 stripes
(S = 5592406) for several row pitches (bytes between consecutive shard rows of a stripe) and a
row-major layout (row i of every stripe adjacent).  One process, us per launch, median of 5.

    python tools/pitch_probe.py [reps]
"""
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chubaofs_amd import reedsolomon  # noqa: E402

K, M, S, NST = 12, 4, 5592406, 8
TOTAL = K + M
R256 = (S + 255) // 256 * 256
R4K = (S + 4095) // 4096 * 4096


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    enc = reedsolomon.New(K, M, device=0)
    st = torch.cuda.Stream(device=dev)
    layouts = [("pitch 256-round (bench)", R256, False), ("pitch 4K-round", R4K, False),
               ("4K-round + 256", R4K + 256, False), ("4K-round + 1K", R4K + 1024, False),
               ("4K-round + 2K", R4K + 2048, False), ("4K-round + 4K+256", R4K + 4096 + 256, False),
               ("256-round + 64", R256 + 64, False), ("row-major, 256-round", R256, True)]
    for name, pitch, rowmajor in layouts:
        buf = torch.randint(0, 256, (NST * TOTAL * pitch + 4096,), dtype=torch.uint8, device=dev)
        base = (buf.data_ptr() + 255) // 256 * 256
        if rowmajor:
            ptrs = [base + (i * NST + s) * pitch for s in range(NST) for i in range(TOTAL)]
        else:
            ptrs = [base + (s * TOTAL + i) * pitch for s in range(NST) for i in range(TOTAL)]
        ptrs = (ctypes.c_void_p * len(ptrs))(*ptrs)
        enc.encode_batch(ptrs, S, NST, stream=st)
        enc.reconstruct_batch(ptrs, S, NST, [0, 1, 2, 3], stream=st)
        torch.cuda.synchronize()

        def run(kind):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for i in range(reps):
                if kind == "E" or i % 2 == 0:
                    enc.encode_batch(ptrs, S, NST, stream=st)
                else:
                    enc.reconstruct_batch(ptrs, S, NST, [0, 1, 2, 3], stream=st)
            e1.record(st)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / reps * 1e3

        run("A")  # settle
        res = {k: statistics.median(run(k) for _ in range(5)) for k in ("E", "A")}
        gbs = {k: TOTAL * S * NST / (v * 1e-6) / 1e9 for k, v in res.items()}
        print(f"{name:26s} pitch {pitch:8d}  E {res['E']:7.1f} us ({gbs['E'] / 80:5.1f}%)  "
              f"A {res['A']:7.1f} us ({gbs['A'] / 80:5.1f}%)", flush=True)
        del buf


if __name__ == "__main__":
    main()
