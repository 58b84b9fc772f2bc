"""C4's AZ-local repair (EC6P10L2, 48 blobs of 4 MiB: the local stripe of AZ 0, (8, 1), shard 0 lost)
through cfsec_ec_reconstruct_batch: synchronous wall time per call (median) and device time per
asynchronous call (HIP event pairs, back-to-back), rebuilt rows checked.  CFSEC_LIB_PATH picks a
variant library (A/B of the k = 8, m = 1 product's lookahead)."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from chubaofs_amd import _lib, codemode as cm, ec  # noqa: E402
from chubaofs_amd._shards import BatchMarshal  # noqa: E402

torch.cuda.set_device(0)
t4 = cm.GetTactic(cm.EC6P10L2)
tot4, S4, nb4 = t4.N + t4.M + t4.L, 699051, 48
e4 = ec.NewEncoder(ec.Config(CodeMode=t4, EnableVerify=False), device=0)
bufs = [torch.randint(0, 256, (nb4, tot4, S4), dtype=torch.uint8, device="cuda") for _ in range(3)]
st4 = (ctypes.c_int * nb4)()
for b in bufs:
    bm = BatchMarshal([[b[s, i] for i in range(tot4)] for s in range(nb4)], tot4)
    _lib.check(e4._L.cfsec_ec_encode_batch(e4._h, bm.arr, tot4, nb4, bm.mem, st4))
torch.cuda.synchronize()
idx0, _, _ = t4.LocalStripeInAZ(0)
gold = [b[:, idx0[0]].clone() for b in bufs]
lbms = [BatchMarshal([[b[s, i] for i in idx0] for s in range(nb4)], len(idx0)) for b in bufs]
bad = (ctypes.c_int * nb4)(*([0] * nb4))
off = (ctypes.c_int * (nb4 + 1))(*range(nb4 + 1))
stream = torch.cuda.Stream()
flags = torch.zeros(nb4, dtype=torch.int32, device="cuda")


def sync_call(i):
    lbm = lbms[i % 3]
    _lib.check(e4._L.cfsec_ec_reconstruct_batch(e4._h, lbm.arr, len(idx0), nb4, bad, off, 1, lbm.mem, st4))


def async_call(i):
    lbm = lbms[i % 3]
    _lib.check(e4._L.cfsec_ec_reconstruct_batch_async(e4._h, lbm.arr, len(idx0), nb4, bad, off, 1, st4,
                                                      flags.data_ptr(), None, stream.cuda_stream))


for i in range(10):
    sync_call(i)
ts = []
for i in range(300):
    t0 = time.perf_counter()
    sync_call(i)
    ts.append(time.perf_counter() - t0)
ts.sort()
for i in range(10):
    async_call(i)
torch.cuda.synchronize()
evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(300)]
for i, (a, b) in enumerate(evs):
    a.record(stream)
    async_call(i)
    b.record(stream)
torch.cuda.synchronize()
dev = sorted(a.elapsed_time(b) * 1e3 for a, b in evs)
for k, b in enumerate(bufs):
    assert torch.equal(b[:, idx0[0]], gold[k]), "rebuilt rows differ"
alg = 9 * S4 * nb4
print(f"sync median {ts[150] * 1e6:7.1f} us ({alg / ts[150] / 8e12:.4f} of 8 TB/s)  "
      f"async device median {dev[150]:7.1f} us ({alg / dev[150] * 1e6 / 8e12:.4f})", flush=True)
