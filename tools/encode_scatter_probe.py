"""Encode batches with every shard at its own address against the same batch in one buffer
(cfsec_ec_encode_batch_async, HIP events per call, back to back): EC12P4 8 x 64 MiB blobs and
EC16P20L2 64 x 4 MiB blobs; parity checked against the contiguous run's (dev probe, round 4)."""
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
stream = torch.cuda.Stream()
reps = int(os.environ.get("REPS", "20"))
for mode, S, nb in ((cm.EC12P4, 5592406, 8), (cm.EC16P20L2, 262144, 64)):
    t = cm.GetTactic(mode)
    tot, N = t.N + t.M + t.L, t.N
    e = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=False), device=0)
    gold = torch.randint(0, 256, (nb, tot, S), dtype=torch.uint8, device="cuda")
    st = (ctypes.c_int * nb)()
    fl = torch.zeros(nb, dtype=torch.int32, device="cuda")
    bm = BatchMarshal([[gold[s, i] for i in range(tot)] for s in range(nb)], tot)
    _lib.check(e._L.cfsec_ec_encode_batch(e._h, bm.arr, tot, nb, bm.mem, st))
    torch.cuda.synchronize()
    rnd = random.Random(3)
    slot = (S + 255) // 256 * 256 + 4096
    pool = torch.empty(nb * tot * slot + 4096, dtype=torch.uint8, device="cuda")
    perm = list(range(nb * tot))
    rnd.shuffle(perm)
    views = [[None] * tot for _ in range(nb)]
    for b in range(nb):
        for i in range(tot):
            o = perm[b * tot + i] * slot + 256 * rnd.randrange(16)
            views[b][i] = pool[o:o + S]
            views[b][i].copy_(gold[b, i])
    for kind in ("contiguous", "scattered", "contiguous", "scattered"):
        if kind == "contiguous":
            w = gold.clone()
            m = BatchMarshal([[w[s, i] for i in range(tot)] for s in range(nb)], tot)
        else:
            m = BatchMarshal(views, tot)

        def call():
            _lib.check(e._L.cfsec_ec_encode_batch_async(e._h, m.arr, tot, nb, st, fl.data_ptr(), None,
                                                          stream.cuda_stream))
        for _ in range(3):
            call()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            call()
        e1.record(stream)
        torch.cuda.synchronize()
        if kind == "scattered":
            for b in range(nb):
                for i in range(N, tot):
                    assert torch.equal(views[b][i], gold[b, i]), (mode, b, i)
        print(f"{cm.GetTactic(mode).N}+{t.M}+{t.L} {kind:11s}: {e0.elapsed_time(e1) * 1e3 / reps:8.1f} us per call", flush=True)
    del gold, pool, views
