"""Round-5 reproduction of round 4's false ErrVerify (What's weak #1).

C5's tasklet (EC16P20L2, 64 bids x 262,144 B, erased {0, 1, 16, 17}, Reconstruct + Verify) with every
shard at its own address (the bench's scattered pool), repaired over and over on S streams at once
(S = 1: the control).  Every call gets its own flag row, so a false Verify is pinned to the call
that produced it; afterwards the rebuilt rows are compared with the golden ones.

    CFSEC_LIB_PATH=<lib> python tools/r5_stale_dma_probe.py --streams 2 --iters 2000

Prints one JSON line: calls, calls with a flag set, the raw flag words of the first failures (a
CFSEC_BS_DEBUG_FLAGS=1 library writes 0x80000000 | compared row << 24 | column tile), rows ok.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from chubaofs_amd import _lib, codemode as cm, ec  # noqa: E402
from chubaofs_amd._shards import BatchMarshal  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--iters", type=int, default=2000)
    ap.add_argument("--bids", type=int, default=64)
    ap.add_argument("--layout", default="scattered", choices=["scattered", "affine"])
    ap.add_argument("--procs", type=int, default=1, help="processes sharing the GPU (each --streams streams)")
    ap.add_argument("--sync-dir", default=None)
    ap.add_argument("--rank", type=int, default=0)
    args = ap.parse_args()
    if args.procs > 1 and args.sync_dir is None:
        return spawn(args)
    dev = torch.device("cuda:0")
    t5 = cm.GetTactic(cm.EC16P20L2)
    n = t5.N + t5.M + t5.L
    S = 262144
    nb = args.bids
    enc = ec.NewEncoder(ec.Config(CodeMode=t5, EnableVerify=False), device=0)
    er = [0, 1, 16, 17]
    bad = (ctypes.c_int * (4 * nb))(*(er * nb))
    off = (ctypes.c_int * (nb + 1))(*range(0, 4 * nb + 1, 4))
    st = (ctypes.c_int * nb)()
    sets = []
    rnd = np.random.default_rng(5)
    for k in range(args.streams):
        g = torch.Generator(device=dev)
        g.manual_seed(100 + k)
        buf = torch.randint(0, 256, (nb, n, S), dtype=torch.uint8, device=dev, generator=g)
        bm = BatchMarshal([[buf[b, i] for i in range(n)] for b in range(nb)], n)
        _lib.check(enc._L.cfsec_ec_encode_batch(enc._h, bm.arr, n, nb, bm.mem, st))
        torch.cuda.synchronize()
        gold = buf.clone()
        if args.layout == "scattered":
            slot = S + 4096
            pool = torch.empty(nb * n * slot + 4096, dtype=torch.uint8, device=dev)
            perm = rnd.permutation(nb * n)
            rows = [[None] * n for _ in range(nb)]
            for b in range(nb):
                for i in range(n):
                    o = int(perm[b * n + i]) * slot + 256 * int(rnd.integers(16))
                    rows[b][i] = pool[o:o + S]
                    rows[b][i].copy_(gold[b, i])
            del buf
        else:
            pool = buf
            rows = [[buf[b, i] for i in range(n)] for b in range(nb)]
        bm = BatchMarshal(rows, n)
        flags = torch.zeros((args.iters, nb), dtype=torch.int32, device=dev)
        sets.append(dict(pool=pool, rows=rows, gold=gold, bm=bm, flags=flags, stream=torch.cuda.Stream(dev)))
    torch.cuda.synchronize()
    if args.sync_dir:  # every process ready before any repairs: their kernels overlap on the GPU
        open(os.path.join(args.sync_dir, f"ready{args.rank}"), "w").close()
        while len([f for f in os.listdir(args.sync_dir) if f.startswith("ready")]) < args.procs:
            time.sleep(0.01)
    for i in range(args.iters):
        for s in sets:
            _lib.check(enc._L.cfsec_ec_reconstruct_batch_async(
                enc._h, s["bm"].arr, n, nb, bad, off, 1, st, s["flags"][i].data_ptr(), None,
                s["stream"].cuda_stream))
            assert list(st) == [0] * nb
    torch.cuda.synchronize()
    out = {"rank": args.rank, "procs": args.procs, "layout": args.layout, "streams": args.streams, "iters": args.iters, "bids": nb,
           "lib": os.environ.get("CFSEC_LIB_PATH", "chubaofs_amd/libcfsec.so"), "per_stream": []}
    for s in sets:
        fl = s["flags"].cpu().numpy().view(np.uint32)
        badcalls = np.nonzero(fl.any(axis=1))[0]
        first = []
        for c in badcalls[:8]:
            bids = np.nonzero(fl[c])[0]
            first.append({"call": int(c), "bids": [int(b) for b in bids[:8]],
                          "words": [hex(int(fl[c, b])) for b in bids[:8]]})
        rows_ok = all(torch.equal(s["rows"][b][i], s["gold"][b, i]) for b in range(nb) for i in range(n))
        out["per_stream"].append({"calls_with_flag": int(len(badcalls)), "bids_flagged": int((fl != 0).sum()),
                                  "first": first, "rows_equal_golden": bool(rows_ok)})
    out["false_verify_calls"] = sum(p["calls_with_flag"] for p in out["per_stream"])
    print(json.dumps(out), flush=True)


def spawn(args):
    """The processes share the GPU (as the bench's N = 2 rehearsal's ranks did); this parent never
    touches it and starts them as children."""
    d = tempfile.mkdtemp(prefix="r5probe")
    cmd = [sys.executable, "-u", os.path.abspath(__file__), "--streams", str(args.streams), "--iters", str(args.iters),
           "--bids", str(args.bids), "--layout", args.layout, "--procs", str(args.procs), "--sync-dir", d]
    ps = [subprocess.Popen(cmd + ["--rank", str(r)], stdout=subprocess.PIPE) for r in range(args.procs)]
    outs = [p.communicate()[0].decode() for p in ps]
    rc = max(p.returncode for p in ps)
    res = [json.loads(o.strip().splitlines()[-1]) for o in outs if o.strip()]
    print(json.dumps({"procs": args.procs, "rc": rc, "false_verify_calls": sum(r["false_verify_calls"] for r in res),
                      "ranks": res}), flush=True)
    return rc


if __name__ == "__main__":
    sys.exit(main() or 0)
