"""Dev tool: isolate what makes the step kernel slower inside bench.py.

Runs the bench's setup with switchable pieces, then times N back-to-back launches of
encode (E), alternating encode/reconstruct (A), in one process, printing us/launch.

    python tools/bench_env.py [N] [setup...]   setup in {randfull, perstripe, clone}
"""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chubaofs_amd import reedsolomon  # noqa: E402

K, M, S, NST = 12, 4, 5592406, 8
TOTAL = K + M
PITCH = (S + 255) // 256 * 256


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    setup = set(sys.argv[2:])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    if "perstripe" in setup:  # exactly bench.py's fill
        batch = torch.zeros((NST, TOTAL, PITCH), dtype=torch.uint8, device=dev)
        for s in range(NST):
            g = torch.Generator(device=dev)
            g.manual_seed(0xCF5EC000 + s)
            batch[s, :K, :S] = torch.randint(0, 256, (K, S), generator=g, device=dev, dtype=torch.uint8)
    else:
        batch = torch.randint(0, 256, (NST, TOTAL, PITCH), dtype=torch.uint8, device=dev)
    base = batch.data_ptr()
    ptrs = (ctypes.c_void_p * (NST * TOTAL))(*[base + i * PITCH for i in range(NST * TOTAL)])
    enc = reedsolomon.New(K, M, device=0)
    st = torch.cuda.Stream(device=dev)
    enc.encode_batch(ptrs, S, NST, stream=st)
    enc.reconstruct_batch(ptrs, S, NST, [0, 1, 2, 3], stream=st)
    torch.cuda.synchronize()
    if "clone" in setup:
        golden = batch.clone()  # noqa: F841
    torch.cuda.synchronize()

    def run(kind, reps):
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

    for rnd in range(3):
        for kind in ("E", "A"):
            print(f"setup={sorted(setup)} round {rnd} {kind}: {run(kind, n):7.1f} us/launch  "
                  f"windows of 20: {[round(run(kind, 20), 1) for _ in range(5)]}", flush=True)


if __name__ == "__main__":
    main()
