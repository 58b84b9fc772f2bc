#!/usr/bin/env python3
"""Host-memory (PCIe-inclusive) rate of the engine: EC12P4 Encode and Reconstruct(erased
{0,1,2,3}) of 64 MiB blobs held in host memory, through the C ABI's CFSEC_MEM_HOST path (the
one the cgo shim uses).  Pageable numpy buffers vs page-locked ones from cfsec_host_alloc.
Prints one JSON line per case: data GB/s (12*S per stripe) and PCIe GB/s (bytes moved over the
link: encode 12S in + 4S out, reconstruct 12S in + 4S out)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from chubaofs_amd import _lib, codemode as cm, ec  # noqa: E402

K, M = 12, 4
S = (64 << 20) // K + 1  # 5,592,406 (common/ec/buf.go:77-81)


def case(pinned: bool, reps: int):
    enc = ec.NewEncoder(ec.Config(CodeMode=cm.GetTactic(cm.EC12P4), EnableVerify=False))
    buf = _lib.pinned_empty((K + M) * S) if pinned else np.zeros((K + M) * S, np.uint8)
    buf[:K * S] = np.random.default_rng(1).integers(0, 256, K * S, dtype=np.uint8)
    shards = [buf[i * S:(i + 1) * S] for i in range(K + M)]  # ec.Buffer layout
    enc.Encode(shards)
    want = [s.copy() for s in shards[:4]]
    t0 = time.perf_counter()
    for _ in range(reps):
        enc.Encode(shards)
    t_enc = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    for _ in range(reps):
        enc.Reconstruct(shards, [0, 1, 2, 3])
    t_rec = (time.perf_counter() - t0) / reps
    assert all(np.array_equal(a, b) for a, b in zip(shards[:4], want))
    out = {"case": "pinned (cfsec_host_alloc)" if pinned else "pageable", "shard_size": S}
    for name, t in (("encode", t_enc), ("reconstruct", t_rec)):
        out[name + "_ms"] = round(t * 1e3, 3)
        out[name + "_data_GBps"] = round(K * S / t / 1e9, 2)
        out[name + "_pcie_GBps"] = round((K + M) * S / t / 1e9, 2)
    print(json.dumps(out), flush=True)


def case_zero_copy(reps: int):
    """Pinned host pointers handed to the kernels as device pointers (CFSEC_MEM_DEVICE): the GF
    kernel reads and writes host memory over PCIe directly, no staging copies."""
    import ctypes
    L = _lib.lib()
    h = ctypes.c_void_p()
    _lib.check(L.cfsec_rs_new(K, M, -1, ctypes.byref(h)))
    buf = _lib.pinned_empty((K + M) * S)
    buf[:K * S] = np.random.default_rng(1).integers(0, 256, K * S, dtype=np.uint8)
    base = buf.ctypes.data
    arr = (_lib.Shard * (K + M))(*[_lib.Shard(base + i * S, S, S) for i in range(K + M)])
    _lib.check(L.cfsec_rs_encode(h, arr, K + M, _lib.MEM_DEVICE, None))
    want = buf[K * S:].copy()
    buf[K * S:] = 0
    t0 = time.perf_counter()
    for _ in range(reps):
        _lib.check(L.cfsec_rs_encode(h, arr, K + M, _lib.MEM_DEVICE, None))
    t = (time.perf_counter() - t0) / reps
    assert np.array_equal(buf[K * S:], want)
    L.cfsec_rs_free(h)
    print(json.dumps({"case": "pinned zero-copy (kernel on host pointers)", "shard_size": S,
                      "encode_ms": round(t * 1e3, 3), "encode_data_GBps": round(K * S / t / 1e9, 2),
                      "encode_pcie_GBps": round((K + M) * S / t / 1e9, 2)}), flush=True)


if __name__ == "__main__":
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    case(False, reps)
    case(True, reps)
    case_zero_copy(reps)
