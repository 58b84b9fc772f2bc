"""Host-side time of the synchronous batch calls of bench.py's C4 / C5 configs (dev tool):
CFSEC_HOST_TIMING=1 python tools/host_timing.py 2> timing.txt -- wall time per call on stdout, the
library's per-phase times on stderr."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from chubaofs_amd import _lib, codemode as cm, ec  # noqa: E402
from chubaofs_amd._shards import BatchMarshal  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(0)


def run(name, fn, n=20):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        sys.stderr.write(f"--- {name}\n")
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e6)
    ts.sort()
    print(f"{name:28s} wall median {ts[n // 2]:8.1f} us  min {ts[0]:8.1f} us", flush=True)


t5 = cm.GetTactic(cm.EC16P20L2)
tot5, S5, nb5 = t5.N + t5.M + t5.L, 262144, 64
e5 = ec.NewEncoder(ec.Config(CodeMode=t5, EnableVerify=False), device=0)
b5 = torch.randint(0, 256, (nb5, tot5, S5), dtype=torch.uint8, device=dev)
bm5 = BatchMarshal([[b5[s, i] for i in range(tot5)] for s in range(nb5)], tot5)
st5 = (ctypes.c_int * nb5)()
_lib.check(e5._L.cfsec_ec_encode_batch(e5._h, bm5.arr, tot5, nb5, bm5.mem, st5))
bad5 = (ctypes.c_int * (4 * nb5))(*([0, 1, 16, 17] * nb5))
off5 = (ctypes.c_int * (nb5 + 1))(*range(0, 4 * nb5 + 1, 4))
run("C5 reconstruct_batch", lambda: _lib.check(e5._L.cfsec_ec_reconstruct_batch(e5._h, bm5.arr, tot5, nb5, bad5, off5,
                                                                                  1, bm5.mem, st5)))
assert list(st5) == [0] * nb5

t4 = cm.GetTactic(cm.EC6P10L2)
tot4, S4, nb4 = t4.N + t4.M + t4.L, 699051, 48
e4 = ec.NewEncoder(ec.Config(CodeMode=t4, EnableVerify=False), device=0)
b4 = torch.randint(0, 256, (nb4, tot4, S4), dtype=torch.uint8, device=dev)
bm4 = BatchMarshal([[b4[s, i] for i in range(tot4)] for s in range(nb4)], tot4)
st4 = (ctypes.c_int * nb4)()
run("C4 encode_batch", lambda: _lib.check(e4._L.cfsec_ec_encode_batch(e4._h, bm4.arr, tot4, nb4, bm4.mem, st4)))
idx0, _, _ = t4.LocalStripeInAZ(0)
lbm = BatchMarshal([[b4[s, i] for i in idx0] for s in range(nb4)], len(idx0))
bad = (ctypes.c_int * nb4)(*([0] * nb4))
off = (ctypes.c_int * (nb4 + 1))(*range(nb4 + 1))
run("C4 local reconstruct_batch", lambda: _lib.check(e4._L.cfsec_ec_reconstruct_batch(e4._h, lbm.arr, len(idx0), nb4, bad,
                                                                                        off, 1, lbm.mem, st4)))

# asynchronous forms: wall time of the enqueue alone (a sync after each call, outside the timing)
stream = torch.cuda.Stream()
fl = torch.zeros(64, dtype=torch.int32, device=dev)


def timed_async(name, fn, n=20):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        sys.stderr.write(f"--- {name}\n")
        t0 = time.perf_counter()
        fn()
        ts.append((time.perf_counter() - t0) * 1e6)
        torch.cuda.synchronize()
    ts.sort()
    print(f"{name:28s} enqueue median {ts[n // 2]:8.1f} us  min {ts[0]:8.1f} us", flush=True)


timed_async("C5 reconstruct_batch_async", lambda: _lib.check(e5._L.cfsec_ec_reconstruct_batch_async(
    e5._h, bm5.arr, tot5, nb5, bad5, off5, 1, st5, fl.data_ptr(), None, stream.cuda_stream)))
timed_async("C4 local reconstruct_async", lambda: _lib.check(e4._L.cfsec_ec_reconstruct_batch_async(
    e4._h, lbm.arr, len(idx0), nb4, bad, off, 1, st4, fl.data_ptr(), None, stream.cuda_stream)))
timed_async("C4 encode_batch_async", lambda: _lib.check(e4._L.cfsec_ec_encode_batch_async(
    e4._h, bm4.arr, tot4, nb4, st4, None, None, stream.cuda_stream)))
