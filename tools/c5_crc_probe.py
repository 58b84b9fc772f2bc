"""C5's tasklet (EC16P20L2, 64 bids x S = 262,144, erased {0, 1, 16, 17}) through
cfsec_ec_reconstruct_batch_async with and without the rebuilt shards' checksums: device time per
call from HIP events (back-to-back calls), every bid's words against zlib (CFSEC_BS_REPAIR_CRC=1 / 2:
the repair-pass checksum forms).  Run under
rocprofv3 --kernel-trace --stats to see the launches one call makes."""
import ctypes
import os
import sys
import zlib

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from chubaofs_amd import codemode as cm, ec  # noqa: E402
from chubaofs_amd import _lib  # noqa: E402
from chubaofs_amd._shards import BatchMarshal  # noqa: E402

torch.cuda.set_device(0)
t = cm.GetTactic(cm.EC16P20L2)
tot, S, nb = t.N + t.M + t.L, 262144, 64
e = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=False), device=0)
buf = torch.randint(0, 256, (nb, tot, S), dtype=torch.uint8, device="cuda")
bm = BatchMarshal([[buf[s, i] for i in range(tot)] for s in range(nb)], tot)
st = (ctypes.c_int * nb)()
_lib.check(e._L.cfsec_ec_encode_batch(e._h, bm.arr, tot, nb, bm.mem, st))
torch.cuda.synchronize()
gold = buf.clone()
er = [0, 1, 16, 17]
bad = (ctypes.c_int * (4 * nb))(*(er * nb))
off = (ctypes.c_int * (nb + 1))(*range(0, 4 * nb + 1, 4))
flags = torch.zeros(nb, dtype=torch.int32, device="cuda")
words = torch.zeros(nb * tot, dtype=torch.int32, device="cuda")
stream = torch.cuda.Stream()


def call(crc):
    cw = ctypes.c_void_p(words.data_ptr()) if crc else None
    _lib.check(e._L.cfsec_ec_reconstruct_batch_async(e._h, bm.arr, tot, nb, bad, off, 1, st, flags.data_ptr(), cw,
                                                      stream.cuda_stream))


reps = int(os.environ.get("C5_REPS", "50"))
for crc in (False, True, False, True):
    buf[:, er].zero_()
    for _ in range(5):
        call(crc)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        call(crc)
    e1.record(stream)
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / reps
    assert list(st) == [0] * nb and not flags.any().item() and torch.equal(buf, gold)
    print(f"crcs={crc}: {us:8.1f} us per call", flush=True)
if os.environ.get("C5_NOCHECK"):  # timing probes of deliberately wrong-word variants
    sys.exit(0)
words.zero_()
torch.cuda.synchronize()
call(True)
torch.cuda.synchronize()
w = words.cpu().numpy().view("uint32").reshape(nb, tot)
h = gold.cpu().numpy()
for b in range(nb):
    for i in range(tot):
        assert int(w[b, i]) == (zlib.crc32(h[b, i].tobytes()) & 0xFFFFFFFF if i in er else 0), (b, i)
print(f"all {nb} bids: rebuilt rows equal the golden, checksums equal zlib")
