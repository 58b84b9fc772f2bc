"""An ec mode's put batch through cfsec_ec_encode_batch_async with and without every shard's checksum
(device time per call from HIP events, back-to-back calls); the words of every bid checked against zlib.
  python tools/lrc_crc_probe.py EC6P6L9 [S] [bids]      (CFSEC_BS_CRC=0: the product + separate pass)"""
import ctypes
import os
import sys
import zlib

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from chubaofs_amd import codemode as cm, ec  # noqa: E402
from chubaofs_amd import _lib  # noqa: E402
from chubaofs_amd._shards import BatchMarshal  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "EC6P6L9"
S = int(sys.argv[2]) if len(sys.argv) > 2 else 699051
nb = int(sys.argv[3]) if len(sys.argv) > 3 else 48
torch.cuda.set_device(0)
t = cm.GetTactic(getattr(cm, mode))
tot = t.N + t.M + t.L
e = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=False), device=0)
bufs = [torch.randint(0, 256, (nb, tot, S), dtype=torch.uint8, device="cuda") for _ in range(3)]
bms = [BatchMarshal([[b[s, i] for i in range(tot)] for s in range(nb)], tot) for b in bufs]
st = (ctypes.c_int * nb)()
words = torch.zeros(nb * tot, dtype=torch.int32, device="cuda")
stream = torch.cuda.Stream()


def call(i, crc):
    cw = ctypes.c_void_p(words.data_ptr()) if crc else None
    _lib.check(e._L.cfsec_ec_encode_batch_async(e._h, bms[i % 3].arr, tot, nb, st, None, cw, stream.cuda_stream))


for crc in (False, True, False, True):
    for i in range(6):
        call(i, crc)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for i in range(20):
        call(i, crc)
    e1.record(stream)
    torch.cuda.synchronize()
    print(f"{mode} S={S} bids={nb} crcs={crc}: {e0.elapsed_time(e1) * 1e3 / 20:8.1f} us per call", flush=True)
call(0, True)
torch.cuda.synchronize()
w = words.cpu().numpy().view("uint32").reshape(nb, tot)
h = bufs[0].cpu().numpy()
for b in range(nb):
    for i in range(tot):
        assert int(w[b, i]) == zlib.crc32(h[b, i].tobytes()) & 0xFFFFFFFF, (b, i)
print(f"all {nb} bids: {tot} checksums each equal zlib")
