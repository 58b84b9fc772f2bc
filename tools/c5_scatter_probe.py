"""C5's tasklet (EC16P20L2, 64 bids x S = 262,144, erased {0, 1, 16, 17}) with every shard at its
own address -- blobnode's layout, a bid assembled from per-vuid ShardsBuf buffers
(work_shard_recover.go:711-716) -- against the same tasklet in one [bids, 38, S] buffer: device
time per cfsec_ec_reconstruct_batch_async call (HIP events, back-to-back calls), results checked
against the golden rows (dev probe, round 4)."""
import ctypes
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from chubaofs_amd import codemode as cm, ec  # noqa: E402
from chubaofs_amd import _lib  # noqa: E402
from chubaofs_amd._shards import BatchMarshal  # noqa: E402

torch.cuda.set_device(0)
t = cm.GetTactic(cm.EC16P20L2)
tot, S, nb = t.N + t.M + t.L, 262144, 64
e = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=False), device=0)
gold = torch.randint(0, 256, (nb, tot, S), dtype=torch.uint8, device="cuda")
bm = BatchMarshal([[gold[s, i] for i in range(tot)] for s in range(nb)], tot)
st = (ctypes.c_int * nb)()
_lib.check(e._L.cfsec_ec_encode_batch(e._h, bm.arr, tot, nb, bm.mem, st))
torch.cuda.synchronize()
er = [0, 1, 16, 17]
bad = (ctypes.c_int * (4 * nb))(*(er * nb))
off = (ctypes.c_int * (nb + 1))(*range(0, 4 * nb + 1, 4))
flags = torch.zeros(nb, dtype=torch.int32, device="cuda")
stream = torch.cuda.Stream()

# scattered: shard (b, i) in slot perm[b * tot + i] of a pool, slots S + 4 KiB apart plus a random
# multiple of 256 B, so no two rows of a bid and no two bids share a stride
rnd = random.Random(7)
slot = S + 4096
pool = torch.empty(nb * tot * slot + (1 << 20), dtype=torch.uint8, device="cuda")
perm = list(range(nb * tot))
rnd.shuffle(perm)
views = [[None] * tot for _ in range(nb)]
for b in range(nb):
    for i in range(tot):
        o = perm[b * tot + i] * slot + 256 * rnd.randrange(16)
        views[b][i] = pool[o:o + S]
        views[b][i].copy_(gold[b, i])
work = {"contiguous": gold.clone(), "scattered": views}


def marshal(kind):
    if kind == "contiguous":
        w = work[kind]
        return BatchMarshal([[w[s, i] for i in range(tot)] for s in range(nb)], tot)
    return BatchMarshal(views, tot)


def check(kind):
    for b in range(nb):
        for i in er:
            got = work[kind][b, i] if kind == "contiguous" else views[b][i]
            assert torch.equal(got, gold[b, i]), (kind, b, i)


reps = int(os.environ.get("C5_REPS", "30"))
for kind in ("contiguous", "scattered", "contiguous", "scattered"):
    m = marshal(kind)

    def call():
        _lib.check(e._L.cfsec_ec_reconstruct_batch_async(e._h, m.arr, tot, nb, bad, off, 1, st, flags.data_ptr(),
                                                          None, stream.cuda_stream))
    for b in range(nb):
        for i in er:
            (work[kind][b, i] if kind == "contiguous" else views[b][i]).zero_()
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    check(kind)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        call()
    e1.record(stream)
    torch.cuda.synchronize()
    assert list(st) == [0] * nb and not flags.any().item()
    print(f"{kind:11s}: {e0.elapsed_time(e1) * 1e3 / reps:8.1f} us per call", flush=True)
