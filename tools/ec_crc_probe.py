"""ec batch encode with shard checksums (cfsec_ec_encode_batch_async + crcs) on EC12P4, 8 stripes of
64 MiB blobs in one pitched buffer, device time per call from HIP events (back-to-back calls), and the
words of stripe 0 against zlib.  Run once with CFSEC_BATCH_FUSED_CRC=0 (product + separate CRC pass)
and once without (fused product + CRC kernel) for the A/B."""
import ctypes
import os
import sys
import zlib

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from chubaofs_amd import _lib, codemode as cm, ec  # noqa: E402
from chubaofs_amd._shards import BatchMarshal  # noqa: E402

torch.cuda.set_device(0)
t = cm.GetTactic(cm.EC12P4)
n, S, nst = t.N + t.M, 5592406, 8
pitch = (S + 255) // 256 * 256
e = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=False), device=0)
buf = torch.randint(0, 256, (nst, n, pitch), dtype=torch.uint8, device="cuda")
bm = BatchMarshal([[buf[s, i, :S] for i in range(n)] for s in range(nst)], n)
st = (ctypes.c_int * nst)()
words = torch.zeros(nst * n, dtype=torch.int32, device="cuda")
stream = torch.cuda.Stream()


def call(crc):
    cw = ctypes.c_void_p(words.data_ptr()) if crc else None
    _lib.check(e._L.cfsec_ec_encode_batch_async(e._h, bm.arr, n, nst, st, None, cw, stream.cuda_stream))


for crc in (False, True):
    for _ in range(5):
        call(crc)
    torch.cuda.synchronize()
    reps = 30
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        call(crc)
    e1.record(stream)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    print(f"fused={os.environ.get('CFSEC_BATCH_FUSED_CRC', '1')} crcs={crc}: {us:8.1f} us per call "
          f"({16 * S * nst / us / 1e3 / 8000 * 100:5.1f} % of 8 TB/s on the 16 S per stripe)", flush=True)
w = words.cpu().numpy().view("uint32").reshape(nst, n)
h = buf[0, :, :S].cpu().numpy()
for i in range(n):
    assert int(w[0, i]) == zlib.crc32(h[i].tobytes()) & 0xFFFFFFFF, i
print("stripe 0 checksums equal zlib")
