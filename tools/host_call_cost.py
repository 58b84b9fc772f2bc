"""Host cost of one asynchronous batch call (C4's put batch: EC6P10L2, 48 bids x 699,051 B, device
memory): wall time of the call on the host while the GPU is held busy by a spin kernel queued ahead
(so no call waits for the device), with and without checksum words; CFSEC_HOST_TIMING=1 prints the
library's own phase timers for a few calls.
  python tools/host_call_cost.py [mode] [S] [bids]"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from chubaofs_amd import codemode as cm, ec  # noqa: E402
from chubaofs_amd._shards import BatchMarshal  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "EC6P10L2"
S = int(sys.argv[2]) if len(sys.argv) > 2 else 699051
nb = int(sys.argv[3]) if len(sys.argv) > 3 else 48
torch.cuda.set_device(0)
t = cm.GetTactic(getattr(cm, mode))
tot = t.N + t.M + t.L
e = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=False), device=0)
p = (S + 255) // 256 * 256
buf = torch.randint(0, 256, (nb, tot, p), dtype=torch.uint8, device="cuda")
bm = BatchMarshal([[buf[s, i, :S] for i in range(tot)] for s in range(nb)], tot)
st = (ctypes.c_int * nb)()
words = torch.zeros(nb * tot, dtype=torch.int32, device="cuda")
stream = torch.cuda.Stream()
fn = e._L.cfsec_ec_encode_batch_async
cw = ctypes.c_void_p(words.data_ptr())
sp = stream.cuda_stream
for crc in (False, True):
    w = cw if crc else None
    for _ in range(4):
        fn(e._h, bm.arr, tot, nb, st, None, w, sp)
    torch.cuda.synchronize()
    with torch.cuda.stream(stream):
        torch.cuda._sleep(int(2e8))  # device spin: the calls below are enqueued behind it
    n = 48  # fewer than the library's 64 workspaces: no call waits for the device
    t0 = time.perf_counter()
    for _ in range(n):
        fn(e._h, bm.arr, tot, nb, st, None, w, sp)
    dt = (time.perf_counter() - t0) / n
    torch.cuda.synchronize()
    # as the bench times them: back to back, an event pair around each call
    m = 200
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(m)]
    t0 = time.perf_counter()
    for i in range(m):
        evs[i][0].record(stream)
        fn(e._h, bm.arr, tot, nb, st, None, w, sp)
        evs[i][1].record(stream)
    torch.cuda.synchronize()
    host = (time.perf_counter() - t0) / m
    pair = sum(a.elapsed_time(b) for a, b in evs) / m * 1e3
    wall = evs[0][0].elapsed_time(evs[-1][1]) / m * 1e3
    print(f"{mode} S={S} bids={nb} crcs={crc}: host {dt * 1e6:7.1f} us per call with the device busy; back to back: "
          f"event pair {pair:7.1f} us, first-to-last {wall:7.1f} us, host loop {host * 1e6:7.1f} us per call", flush=True)
