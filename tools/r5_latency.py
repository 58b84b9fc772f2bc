"""Where a Python caller's device-memory ReconstructData call spends its time:
Marshal (the cfsec_shard vector from torch tensors), the ctypes call itself (the engine, which ends
synchronously), and torch.cuda.synchronize -- medians over repeated calls, EC6P6 / EC12P4 segments
with data shards {0, 1} bad, the bench's segment_reconstruct_data shape."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from chubaofs_amd import _lib, codemode as cm, ec  # noqa: E402
from chubaofs_amd._shards import Marshal, stream_ptr  # noqa: E402


def med(fn, n=200):
    for _ in range(5):
        fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return round(ts[n // 2] * 1e6, 1)


out = {}
for name, mode in (("EC6P6", cm.EC6P6), ("EC12P4", cm.EC12P4)):
    t = cm.GetTactic(mode)
    n = t.N + t.M
    enc = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=False), device=0)
    for seg in (4096, 65536):
        segs = [torch.randint(0, 256, (seg,), dtype=torch.uint8, device="cuda") for _ in range(n)]
        enc.Encode(segs)
        torch.cuda.synchronize()
        bad = [0, 1]
        badarr = (ctypes.c_int * 2)(*bad)
        r = {}
        r["python_api_us"] = med(lambda: (enc.ReconstructData(list(segs), bad), torch.cuda.synchronize()))
        r["marshal_us"] = med(lambda: Marshal(list(segs)))
        m = Marshal(list(segs))
        sp = stream_ptr(None, segs[0])
        r["stream_ptr_us"] = med(lambda: stream_ptr(None, segs[0]))
        r["ctypes_call_us"] = med(lambda: enc._L.cfsec_ec_reconstruct_data(enc._h, m.ptr(), m.n, badarr, 2, m.mem, sp))
        r["torch_sync_us"] = med(lambda: torch.cuda.synchronize())
        out[f"{name}_{seg}"] = r
print(json.dumps(out), flush=True)
