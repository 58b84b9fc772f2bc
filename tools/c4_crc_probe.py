"""C4's put batch (EC6P10L2, 48 blobs x S = 699,051) through cfsec_ec_encode_batch_async with and
without all 18 checksums per blob: device time per call from HIP events (back-to-back calls), the
words of blob 0 against zlib.  CFSEC_BATCH_FUSED_CRC=0 runs the checksums as the separate pass
(A/B of the fused 6 x (10 + 2) encode + CRC kernel); CFSEC_CRC_LDS12=0 the round-5 v_perm form of it.
Every blob's parity and 18 words are checked after the timing.""" 
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
t = cm.GetTactic(cm.EC6P10L2)
tot, S, nb = t.N + t.M + t.L, 699051, 48
e = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=False), device=0)
bufs = [torch.randint(0, 256, (nb, tot, S), dtype=torch.uint8, device="cuda") for _ in range(3)]
bms = [BatchMarshal([[b[s, i] for i in range(tot)] for s in range(nb)], tot) for b in bufs]
st = (ctypes.c_int * nb)()
words = torch.zeros(nb * tot, dtype=torch.int32, device="cuda")
stream = torch.cuda.Stream()


def call(i, crc):
    cw = ctypes.c_void_p(words.data_ptr()) if crc else None
    _lib.check(e._L.cfsec_ec_encode_batch_async(e._h, bms[i % 3].arr, tot, nb, st, None, cw, stream.cuda_stream))


reps = int(os.environ.get("C4_REPS", "30"))
for crc in (False, True, False, True):
    for i in range(6):
        call(i, crc)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for i in range(reps):
        call(i, crc)
    e1.record(stream)
    torch.cuda.synchronize()
    print(f"crcs={crc}: {e0.elapsed_time(e1) * 1e3 / reps:8.1f} us per call", flush=True)
    assert list(st) == [0] * nb
call(0, False)
torch.cuda.synchronize()
plain = bufs[0][:, t.N:].clone()
bufs[0][:, t.N:] = 0
torch.cuda.synchronize()  # the zero fill ran on torch's stream, the calls run on `stream`
call(0, True)
torch.cuda.synchronize()
assert torch.equal(bufs[0][:, t.N:], plain), "parity rows of the checksummed call differ from the plain encode"
w = words.cpu().numpy().view("uint32").reshape(nb, tot)
h = bufs[0].cpu().numpy()
for b in range(nb):
    for i in range(tot):
        assert int(w[b, i]) == zlib.crc32(h[b, i].tobytes()) & 0xFFFFFFFF, (b, i)
print(f"all {nb} blobs: parity equal to the plain encode, {tot} checksums each equal zlib")
