"""Dev tool: isolate what makes the step kernel slower inside the bench process.

Times 200 back-to-back EC12P4 encode launches (8 x 64 MiB-blob stripes) for each combination
of {torch-allocated, hipMalloc-allocated} buffer x {torch stream, null stream}, in one process.
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
NBYTES = NST * TOTAL * PITCH

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]


def main():
    dev = torch.device("cuda", 0)
    tbuf = torch.randint(0, 256, (NBYTES,), dtype=torch.uint8, device=dev)
    hptr = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(hptr), NBYTES) == 0
    assert hip.hipMemcpy(hptr, ctypes.c_void_p(tbuf.data_ptr()), NBYTES, 3) == 0  # D2D
    torch.cuda.synchronize()
    enc = reedsolomon.New(K, M, device=0)
    tstream = torch.cuda.Stream(device=dev)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    for rnd in range(2):
        for bname, base in (("torch-buf", tbuf.data_ptr()), ("hipMalloc-buf", hptr.value)):
            ptrs = (ctypes.c_void_p * (NST * TOTAL))(*[base + i * PITCH for i in range(NST * TOTAL)])
            for sname, st in (("torch-stream", tstream), ("null-stream", None)):
                s = tstream if st is not None else torch.cuda.default_stream(dev)
                for _ in range(10):
                    enc.encode_batch(ptrs, S, NST, stream=st)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                for _ in range(n):
                    enc.encode_batch(ptrs, S, NST, stream=st)
                e1.record(s)
                torch.cuda.synchronize()
                us = e0.elapsed_time(e1) / n * 1e3
                print(f"round {rnd} {bname:14s} {sname:13s} {us:7.1f} us/launch  "
                      f"{TOTAL * S * NST / (us * 1e-6) / 1e9:7.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
