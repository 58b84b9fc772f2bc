#!/usr/bin/env python3
"""bench.py -- EC12P4 encode + 4-erasure reconstruct throughput on MI355X.

Workload (BASELINE.json configs[1]/[2], per GPU): batches of `--stripes` EC12P4 stripes of 64 MiB
blobs (shard size S = ceil(64 MiB / 12) = 5,592,406 B), resident in HBM with a 256-B shard pitch.
One step = one pass of the hot path over one batch of each operation:
  1. Encode       (cfsec_rs_encode_batch):      read 12*S, write 4*S per stripe
  2. Reconstruct  erased {0,1,2,3}, the worst-case dense decode
                  (cfsec_rs_reconstruct_batch): read 12*S, write 4*S per stripe
value = data bytes through the engine per second = 2 * 12 * S * stripes * n_gpus / step time
(each operation counts its stripe's 12*S data bytes once).  Multi-GPU: each rank codes its own
stripes (weak scaling, no collective on the data path).

No cache reuse between launches: the GPU holds three batches (3 x 716 MB) and step i encodes batch
i % 3 and reconstructs batch (i + 2) % 3, so between two launches over the same batch at least
1.4 GB of other traffic passes through the 256 MB Infinity Cache -- every launch reads its inputs
from HBM (round 1 alternated the two operations on ONE batch, and each re-read the 179 MB the other
had just written).

Correctness gate (fails a kernel that writes nothing or wrong bytes inside the timed region):
before the timed region, every batch's rows that its first timed operation writes are zeroed
(parity before an encode, rows 0-3 before a reconstruct); after it, every row must equal the
golden codeword (data from the seeded generator, parity from the first encode, which the CPU leg
checks against the klauspost-strategy CPU port on stripe 0).

    python bench.py [--gpus N --steps K --warmup W]

--gpus N > 1 without a torch.distributed environment re-launches this script under
`python -m torch.distributed.run --nproc-per-node N` as a child process (before this process
touches a GPU) and exits with its status.
"""
from __future__ import annotations

import argparse
import ctypes
import csv
import glob
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

K_DATA, M_PARITY = 12, 4
BLOB = 64 << 20
S_DEFAULT = (BLOB + K_DATA - 1) // K_DATA  # 5,592,406 (common/ec/buf.go:77-81)
ERASED = [0, 1, 2, 3]
NBATCH = 3  # batches rotated through the step (no Infinity-Cache reuse between launches)
HBM_PEAK_GBPS = 8000.0  # MI355X spec (MI355X_MICROARCH.md)
CPU_SHARE = 16  # host CPUs leased with one GPU on the bench pool
# Both step launches (encode, reconstruct of {0,1,2,3}) are 12 -> 4 row products on the 4x4-dyadic
# kernel (the lookup-product kernel is 4 % behind on this shape: profiles/r03/bench_lut_ab.txt)
KERNEL = "gf_dy_kernel<12, 4, 4, (cfsec::MatVecMode)0, 0>"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--stripes", type=int, default=8, help="stripes per batch (per GPU per operation)")
    p.add_argument("--shard-size", type=int, default=S_DEFAULT)
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample length")
    p.add_argument("--op-seconds", type=float, default=1.5, help="device time per isolated-operation figure")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-pmc", action="store_true")
    p.add_argument("--no-extra", action="store_true", help="skip the secondary per-operation figures")
    p.add_argument("--graph", action="store_true", help="replay each step as a captured HIP graph")
    p.add_argument("--settle-ms", type=float, default=2000.0, help="untimed load before warmup (clock ramp)")
    p.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    return p.parse_args()


# ----------------------------------------------------------------- multi-rank launch
def spawn_ranks(args) -> int:
    """Run this script as N rank processes under torch.distributed.run (a child process: this
    process never touched a GPU) and return its exit status."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


# ----------------------------------------------------------------- PMC traffic
def _read_counter_csv(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    return rows


def pmc_traffic(args):
    """HBM bytes per launch of the step kernel from rocprofv3 FETCH_SIZE / WRITE_SIZE, one
    counter per pass (MI355X_MICROARCH.md: FETCH_SIZE counts half of a 16-B/lane stream on
    gfx950 -> doubled; both in KiB)."""
    exe = shutil.which("rocprofv3")
    if not exe:
        return None, "rocprofv3 not found"
    vals = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
        cmd = ["timeout", "-s", "KILL", "120", exe, "--pmc", ctr, "--output-format", "csv", "-d", d, "-o", "pmc",
               "--", sys.executable, os.path.abspath(__file__), "--pmc-child", "--steps", "3", "--warmup", "1",
               "--stripes", str(args.stripes), "--shard-size", str(args.shard_size)]
        r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
        if r.returncode != 0:
            return None, f"rocprofv3 --pmc {ctr} failed rc={r.returncode}: {r.stdout[-300:]}"
        per = []
        for row in _read_counter_csv(d):
            name = row.get("Kernel_Name", "")
            if KERNEL.replace(" ", "") in name.replace(" ", "") and row.get("Counter_Name", ctr) == ctr:
                per.append(float(row["Counter_Value"]))
        shutil.rmtree(d, ignore_errors=True)
        if not per:
            return None, f"no {ctr} rows for {KERNEL}"
        vals[ctr] = sum(per) / len(per)
    return (2.0 * vals["FETCH_SIZE"] + vals["WRITE_SIZE"]) * 1024.0, None


# ----------------------------------------------------------------- CPU baseline
def host_cpu_share():
    """CPUs this process may use: the affinity mask, capped by a cgroup v2 CPU quota if one is set
    (the GPU box shows the whole machine in os.cpu_count() but leases a share of it)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    usable = min(aff, quota) if quota else aff
    # the GPU pool leases 16 host CPUs per GPU (its rules: size worker pools to that share, whatever
    # os.cpu_count() or the affinity mask show)
    return {"os_cpu_count": os.cpu_count(), "affinity": aff, "cgroup_quota": quota, "lease_share": CPU_SHARE,
            "usable": min(usable, CPU_SHARE)}


def cpu_baseline(S, seconds, stripe0_host, parity0_gpu):
    """klauspost-strategy restatement (oracle/cpu_simd.c) on the host: EC12P4 encode + 4-erasure
    reconstruct of stripe 0 of the GPU's batch 0, repeated for ~`seconds`, with the reference's
    per-call worker cap (4 with GFNI, else 8; KRS/reedsolomon.go:551-557).  Its parity is also the
    check of the GPU's golden parity for that stripe (the bench's correctness gate)."""
    import numpy as np

    from oracle import oracle as O

    feats = O.simd_features()
    threads = 4 if feats["gfni"] else 8
    data = [np.ascontiguousarray(stripe0_host[i]) for i in range(K_DATA)]
    parity = [np.zeros(S, np.uint8) for _ in range(M_PARITY)]
    full = O.build_matrix(K_DATA, K_DATA + M_PARITY)
    prow = full[K_DATA:]
    err, dec = O.invert(full[4:16])  # survivors 4..15 after erasing {0,1,2,3}
    assert err == 0
    drows = dec[:4]
    survivors = data[4:] + parity
    rebuilt = [np.zeros(S, np.uint8) for _ in range(4)]
    O.simd_code(prow, data, parity, threads)  # warm
    parity_ok = all(np.array_equal(parity[r], parity0_gpu[r]) for r in range(M_PARITY))
    ops, t0 = 0, time.perf_counter()
    kind = 0
    while True:
        kind = O.simd_code(prow, data, parity, threads)
        O.simd_code(drows, survivors, rebuilt, threads)
        ops += 1
        dt = time.perf_counter() - t0
        if dt >= seconds:
            break
    for i in range(4):
        assert np.array_equal(rebuilt[i], data[i]), "CPU baseline reconstruct mismatch"
    value = 2 * K_DATA * S * ops / dt / 1e9
    share = host_cpu_share()
    saturated = cpu_saturated(S, prow, drows, max(2.0, seconds / 2), share["usable"])
    return {
        "value": round(value, 3), "unit": "GB/s", "cores": threads, "kind": "port",
        "sample": (f"EC12P4 encode + erase{{0,1,2,3}} reconstruct of one S={S} stripe x{ops} "
                   f"({dt:.1f}s), klauspost v1.11.7 strategy restated in C "
                   f"({'AVX2 10x4+2x4 tiles' if kind == 1 else 'GFNI tiles'}), {threads} worker threads"),
        "host_cpus": share,
        "features": feats,
        "saturated": saturated,
    }, parity_ok


def cpu_saturated(S, prow, drows, seconds, callers):
    """BASELINE.md's second CPU mode: one single-threaded caller per usable host CPU (affinity
    mask, capped by the cgroup quota and the pool's 16-CPU lease share), each coding its own EC12P4
    stripe (encode + the {0,1,2,3} reconstruct), for ~`seconds`."""
    import threading

    import numpy as np

    from oracle import oracle as O

    callers = max(1, int(callers))
    done = [0] * callers
    stop = time.perf_counter() + seconds

    def worker(w):
        rng = np.random.default_rng(0xCF5EC000 + w)
        data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(K_DATA)]
        parity = [np.zeros(S, np.uint8) for _ in range(M_PARITY)]
        rebuilt = [np.zeros(S, np.uint8) for _ in range(4)]
        O.simd_code(prow, data, parity, 1)
        while time.perf_counter() < stop:
            O.simd_code(prow, data, parity, 1)
            O.simd_code(drows, data[4:] + parity, rebuilt, 1)
            done[w] += 1

    t0 = time.perf_counter()
    threads = [threading.Thread(target=worker, args=(w,)) for w in range(callers)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    dt = time.perf_counter() - t0
    return {"value": round(2 * K_DATA * S * sum(done) / dt / 1e9, 3), "unit": "GB/s", "cores": callers,
            "sample": f"{callers} concurrent single-threaded callers x {sum(done)} stripe passes in {dt:.1f}s"}


# ----------------------------------------------------------------- GPU
GATE_FAILURES = []  # secondary legs whose gate (or anything else) failed: top level of the line + exit status


def leg(name, fn):
    """A secondary leg: its exception is recorded in its field AND in the line's top-level
    `gate_failures`, and makes the run exit non-zero (after the line is printed: the headline stays)."""
    try:
        return fn()
    except Exception as e:  # noqa: BLE001 -- reported in the JSON line, with the traceback on stderr
        import traceback
        traceback.print_exc()
        msg = f"{type(e).__name__}: {e}"
        GATE_FAILURES.append({"leg": name, "error": msg})
        return {"error": msg}


EXIT_GATE_FAILED = 3


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and not args.pmc_child:
        sys.exit(spawn_ranks(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if not args.pmc_child and world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    S, nst = args.shard_size, args.stripes

    traffic, pmc_note = None, "skipped"
    if rank == 0 and world == 1 and not args.no_pmc and not args.pmc_child:
        traffic, pmc_note = pmc_traffic(args)  # before this process touches the GPU

    import torch

    from chubaofs_amd import reedsolomon

    # CFSEC_BENCH_SHARE_DEVICE / CFSEC_BENCH_BACKEND: rehearsal of the N-rank flow on a box with
    # fewer GPUs (ranks share devices round-robin, gloo instead of RCCL, which refuses two ranks on
    # one GPU); the driver's multi-GPU runs use neither
    ndev = torch.cuda.device_count()
    gpu = local_rank % ndev if os.environ.get("CFSEC_BENCH_SHARE_DEVICE") else local_rank
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("CFSEC_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        assert dist.get_world_size() == args.gpus

    total = K_DATA + M_PARITY
    pitch = (S + 255) // 256 * 256
    batch = torch.zeros((NBATCH, nst, total, pitch), dtype=torch.uint8, device=dev)
    for b in range(NBATCH):
        for s in range(nst):  # seeded synthetic data, one generator per stripe
            g = torch.Generator(device=dev)
            g.manual_seed(0xCF5EC000 + (rank * NBATCH + b) * nst + s)
            batch[b, s, :K_DATA, :S] = torch.randint(0, 256, (K_DATA, S), generator=g, device=dev,
                                                     dtype=torch.uint8)
    ptrs = []
    for b in range(NBATCH):
        base = batch[b].data_ptr()
        p = [base + (s * total + i) * pitch for s in range(nst) for i in range(total)]
        ptrs.append((ctypes.c_void_p * len(p))(*p))  # marshalled once, reused by every launch
    enc = reedsolomon.New(K_DATA, M_PARITY, device=dev.index)
    stream = torch.cuda.Stream(device=dev)
    launches = [0]  # launches of the step kernel so far (one per batch call: affine 8-stripe batch)

    def encode(b):
        enc.encode_batch(ptrs[b], S, nst, stream=stream)
        launches[0] += 1

    def reconstruct(b):
        enc.reconstruct_batch(ptrs[b], S, nst, ERASED, stream=stream)
        launches[0] += 1

    step_no = [0]

    def step():
        i = step_no[0]
        encode(i % NBATCH)
        reconstruct((i + 2) % NBATCH)
        step_no[0] += 1

    with torch.cuda.stream(stream):
        for b in range(NBATCH):
            encode(b)  # the golden parity
    torch.cuda.synchronize()

    if args.pmc_child:
        for _ in range(args.warmup + args.steps):
            step()
        torch.cuda.synchronize()
        return

    golden = batch[:, :, :, :S].clone()
    golden_stripe0 = golden[0, 0].cpu().numpy() if rank == 0 else None
    reconstruct(0)  # plans the reconstruct (inversion cache) before any timing or capture
    torch.cuda.synchronize()
    graph = None
    if args.graph:
        # optional: the three steps of one rotation captured into a HIP graph
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            for _ in range(NBATCH):
                step()
        torch.cuda.synchronize()
        assert args.steps % NBATCH == 0, "--graph replays whole rotations: --steps must be a multiple of 3"

    def run_steps(n):
        if graph is None:
            for _ in range(n):
                step()
        else:
            with torch.cuda.stream(stream):
                for _ in range(n // NBATCH):
                    graph.replay()
                    launches[0] += 2 * NBATCH
            step_no[0] += n

    # Settle: after idle the first ~100-200 launches run up to 10 % slower while the clocks ramp
    # (tools/bench_env.py), so the device runs the step for --settle-ms before the W warmup steps.
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < args.settle_ms / 1e3:
        run_steps(NBATCH * 4)
        torch.cuda.synchronize()
    run_steps(args.warmup)
    torch.cuda.synchronize()

    # gate: zero what each batch's first timed operation writes
    first = {}
    for j in range(args.steps):
        i = step_no[0] + j
        first.setdefault(i % NBATCH, "encode")
        first.setdefault((i + 2) % NBATCH, "reconstruct")
    for b, op in first.items():
        if op == "encode":
            batch[b, :, K_DATA:, :].zero_()
        else:
            batch[b, :, ERASED[0]:ERASED[-1] + 1, :].zero_()  # a view: rows 0..3
    torch.cuda.synchronize()

    timed_first = launches[0]
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    run_steps(args.steps)
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    timed_last = launches[0]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    # both step launches are the same 12 -> 4 kernel moving the same algorithmic bytes
    avg_ms = ev0.elapsed_time(ev1) / (2 * args.steps)

    # correctness gate: every row the timed launches wrote is the golden codeword again
    for b in range(NBATCH):
        assert torch.equal(batch[b, :, :, :S], golden[b]), f"batch {b} differs from the golden codeword after the timed steps"
    gate = {"zeroed_before_timed": {str(b): op for b, op in sorted(first.items())}, "rows_equal_golden": True}

    # Strong scaling: the same nst-stripe total split over the ranks -- each codes the
    # first ceil(nst / world) stripes of its batches -- timed like the headline (barrier + sync on both
    # sides, max over ranks).  At N = 1 it is the headline's work; the driver's curve is the weak one.
    per_rank = max(1, -(-nst // world))
    strong_steps = max(NBATCH, args.steps // NBATCH * NBATCH)

    def strong_step(i):
        enc.encode_batch(ptrs[i % NBATCH], S, per_rank, stream=stream)
        enc.reconstruct_batch(ptrs[(i + 2) % NBATCH], S, per_rank, ERASED, stream=stream)

    with torch.cuda.stream(stream):
        for i in range(NBATCH):
            strong_step(i)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    ts0 = time.perf_counter()
    with torch.cuda.stream(stream):
        for i in range(strong_steps):
            strong_step(i)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    st_el = time.perf_counter() - ts0
    if world > 1:
        t = torch.tensor([st_el], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        st_el = float(t.item())
    for b in range(NBATCH):
        assert torch.equal(batch[b, :, :, :S], golden[b]), f"batch {b} differs from the golden codeword (strong run)"
    strong = {"total_stripes": per_rank * world, "stripes_per_gpu": per_rank, "steps": strong_steps,
              "value": round(2 * K_DATA * S * per_rank * world * strong_steps / st_el / 1e9, 2), "unit": "GB/s",
              "ms_per_step": round(st_el / strong_steps * 1e3, 4),
              "note": ("fixed total work (BASELINE configs[2] strong scaling): the 8-stripe batch split over the "
                       "GPUs, same step as the headline; rows checked against the golden codeword afterwards")}

    data_bytes = K_DATA * S * nst
    launch_bytes = (K_DATA + M_PARITY) * S * nst  # algorithmic bytes per launch (read 12S + write 4S)
    achieved = launch_bytes / (avg_ms * 1e-3) / 1e9
    value = 2 * data_bytes * world * args.steps / elapsed / 1e9

    extra = {}
    if not args.no_extra:
        extra = secondary(args, torch, enc, batch, ptrs, stream, S, nst, pitch, dev, launch_bytes, data_bytes)
        del batch, golden
        torch.cuda.empty_cache()
        cpu_here = world == 1 and rank == 0 and not args.no_cpu
        # the secondary legs run after the headline is measured and gated: an exception in one (every
        # rank runs the same code on the same shapes, so it raises on all of them) is recorded in its
        # field instead of costing the job its headline line
        extra["C5_multi_gpu_repair"] = leg("C5_multi_gpu_repair", lambda: multi_gpu_repair(args, torch, dev, rank, world))
        extra["segment_reconstruct_data"] = leg("segment_reconstruct_data", lambda: segment_latency(args, torch, dev, cpu=cpu_here))
        extra["configs"] = leg("configs", lambda: other_configs(args, torch, dev, stream, cpu=cpu_here))
        extra["host_path"] = leg("host_path", lambda: host_path(args, torch, dev, world))

    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return
    cpu = None
    if world == 1 and not args.no_cpu:
        stripe0 = golden_stripe0
        cpu, parity_ok = cpu_baseline(S, args.cpu_seconds, stripe0[:K_DATA], stripe0[K_DATA:])
        assert parity_ok, "GPU golden parity of stripe 0 differs from the CPU port's"
        gate["stripe0_parity_equals_cpu_port"] = True
    out = {
        "metric": "EC12P4 encode + 4-erasure reconstruct data GB/s",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: seeded uniform bytes (torch Generator seed 0xCF5EC000 + stripe), HBM-resident",
        "config": {
            "workload": "EC12P4 Encode then Reconstruct(erased {0,1,2,3}) of 64 MiB-blob stripes",
            "code_mode": "EC12P4", "shard_size": S, "shard_pitch": pitch, "stripes_per_batch": nst,
            "batches_rotated": NBATCH, "erased": ERASED,
            "parallelism": f"stripes sharded over {world} GPU(s), no collective",
            "value_def": "2 * 12 * S * stripes * n_gpus / step time (encode and reconstruct each count the stripe's data once)",
        },
        "roofline": {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": None if traffic is None else int(traffic),
            "kernel": "gf_dy_kernel<12, 4, 4, kStore, 0> (encode and reconstruct launches: both matrices are 4x4-dyadic)",
            "kernel_match": KERNEL,
            "algorithmic_bytes_per_launch": launch_bytes,
            "avg_launch_ms": round(avg_ms, 4),
            "launch_timing": ("HIP event pair on the launch stream around the timed region / launches"
                              + (" (graph replay)" if graph is not None else "")),
            "timed_dispatches": [timed_first, timed_last],
            "timed_dispatches_note": ("0-based indices [first, last) of the timed launches among this process's "
                                      "launches of `kernel`, in dispatch order (tools/timed_region_stats.py)"),
            "traffic_note": pmc_note if traffic is None else "rocprofv3 (2*FETCH_SIZE + WRITE_SIZE)*1024, per launch",
            "cache_note": ("3 batches rotated (step i: encode i%3, reconstruct (i+2)%3): >= 1.4 GB of other traffic "
                           "between two launches over the same batch, so the 256 MB Infinity Cache serves no reuse"),
        },
        "gate": gate,
        "strong_scaling": strong,
        "cpu_baseline": cpu,
    }
    out["gate_failures"] = GATE_FAILURES  # [] when every secondary leg's gate held
    out.update(extra)
    if "stream_copy_GBps" in extra:
        out["roofline"]["measured_peak_GBps"] = extra["stream_copy_GBps"]
        out["roofline"]["frac_of_measured_copy"] = round(achieved / extra["stream_copy_GBps"], 4)
        out["roofline"]["measured_peak_note"] = ("cfsec_stream_copy: a flat float4 non-temporal copy (1 read : 1 write) "
                                                 "on the same rotated batches; the step kernel's 12 : 4 pattern may sit "
                                                 "above or below it")
    elif "device_copy_GBps" in extra:
        out["roofline"]["frac_of_measured_copy"] = round(achieved / extra["device_copy_GBps"], 4)
    print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()
    if GATE_FAILURES:
        print(f"bench: {len(GATE_FAILURES)} secondary gate(s) failed: "
              + "; ".join(f"{g['leg']}: {g['error']}" for g in GATE_FAILURES), file=sys.stderr, flush=True)
        sys.exit(EXIT_GATE_FAILED)


def secondary(args, torch, enc, batch, ptrs, stream, S, nst, pitch, dev, launch_bytes, data_bytes):
    """Per-operation figures outside the timed region: each operation repeated for ~op_seconds of
    device time, rotating over the batches like the step (no cache reuse)."""

    def timed(fn):
        for i in range(6):  # settle after the idle gap of the host-side checks; estimate
            fn(i % NBATCH)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(6):
            fn(i % NBATCH)
        e1.record(stream)
        torch.cuda.synchronize()
        est = max(e0.elapsed_time(e1) / 6, 1e-3)
        n = max(args.steps, int(args.op_seconds * 1e3 / est))
        e0.record(stream)
        for i in range(n):
            fn(i % NBATCH)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n

    rate = lambda nbytes, ms: round(nbytes / (ms * 1e-3) / 1e9, 1)
    frac = lambda nbytes, ms: round(nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)
    out = {}
    enc_ms = timed(lambda b: enc.encode_batch(ptrs[b], S, nst, stream=stream))
    rec_ms = timed(lambda b: enc.reconstruct_batch(ptrs[b], S, nst, ERASED, stream=stream))
    flags = torch.zeros(nst, dtype=torch.int32, device=dev)
    verify_ms = timed(lambda b: enc.verify_batch(ptrs[b], S, nst, flags.data_ptr(), stream=stream))
    assert int(flags.sum().item()) == 0, "Verify failed after the timed region"
    # Encode + crc32.ChecksumIEEE of all 16 shards (access/stream_put.go:249-253), fused into the
    # coding kernel: same algorithmic bytes as the encode
    total = K_DATA + M_PARITY
    crcs = torch.zeros(nst * total, dtype=torch.int32, device=dev)
    crc_ms = timed(lambda b: enc.encode_crc_batch(ptrs[b], S, nst, crcs.data_ptr(), stream=stream))
    # The same through the ec seam access calls (ec.Encoder EncodeBatch with checksums, asynchronous
    # form on the stream): planning + the fused kernel where the group qualifies
    from chubaofs_amd import _lib, codemode as cm, ec
    from chubaofs_amd._shards import BatchMarshal
    e12 = ec.NewEncoder(ec.Config(CodeMode=cm.GetTactic(cm.EC12P4), EnableVerify=False), device=dev.index)
    bms = [BatchMarshal([[batch[b, s, i, :S] for i in range(total)] for s in range(nst)], total) for b in range(NBATCH)]
    est = (ctypes.c_int * nst)()
    ecrc = torch.zeros(nst * total, dtype=torch.int32, device=dev)

    def ec_crc(b):
        _lib.check(e12._L.cfsec_ec_encode_batch_async(e12._h, bms[b].arr, total, nst, est, None,
                                                      ctypes.c_void_p(ecrc.data_ptr()), stream.cuda_stream))

    ec_crc_ms = timed(ec_crc)
    ec_crc(0)
    torch.cuda.synchronize()
    assert list(est) == [0] * nst
    import zlib
    w = ecrc.cpu().numpy().view("uint32").reshape(nst, total)
    for s_ in (0, nst - 1):
        for i in (0, K_DATA, total - 1):
            assert int(w[s_, i]) == zlib.crc32(batch[0, s_, i, :S].cpu().numpy().tobytes()) & 0xFFFFFFFF, "ec seam crc"
    out.update({"ec_seam_encode_crc_ms": round(ec_crc_ms, 4),
                "ec_seam_encode_crc_roofline_frac": frac(launch_bytes, ec_crc_ms)})
    del bms, ecrc
    out.update({
        "encode_data_GBps": rate(data_bytes, enc_ms), "encode_roofline_frac": frac(launch_bytes, enc_ms),
        "reconstruct_data_GBps": rate(data_bytes, rec_ms), "reconstruct_roofline_frac": frac(launch_bytes, rec_ms),
        "verify_data_GBps": rate(data_bytes, verify_ms), "verify_roofline_frac": frac(launch_bytes, verify_ms),
        "encode_crc_data_GBps": rate(data_bytes, crc_ms), "encode_crc_roofline_frac": frac(launch_bytes, crc_ms),
    })
    # Blobnode's write path frames each shard in 64 KiB crc32block blocks and takes the shard's
    # checksum on the way (core/storage/datafile.go:345-373); its read path checks and unframes them
    # (datafile.go:406-426).  All 16 shards of every stripe of a batch in one framing / checking launch.
    from chubaofs_amd import crc32block
    nsh = nst * total
    flen = crc32block.EncodeSize(S)
    fpitch = (flen + 255) // 256 * 256
    framed = torch.empty((NBATCH, nsh, fpitch), dtype=torch.uint8, device=dev)
    unframed = torch.empty((NBATCH, nsh, pitch), dtype=torch.uint8, device=dev)
    fptrs = [(ctypes.c_void_p * nsh)(*[framed[b, i].data_ptr() for i in range(nsh)]) for b in range(NBATCH)]
    uptrs = [(ctypes.c_void_p * nsh)(*[unframed[b, i].data_ptr() for i in range(nsh)]) for b in range(NBATCH)]
    fcrc = torch.zeros(nsh, dtype=torch.int32, device=dev)
    fbad = torch.zeros(nsh, dtype=torch.int32, device=dev)
    blk_enc_ms = timed(lambda b: crc32block.encode_batch(ptrs[b], fptrs[b], S, shard_crcs_ptr=fcrc.data_ptr(),
                                                         stream=stream))
    blk_dec_ms = timed(lambda b: crc32block.decode_batch(fptrs[b], uptrs[b], S, fbad.data_ptr(), stream=stream,
                                                         src_len=fpitch))
    assert bool((fbad == -1).all().item()), "crc32block check failed on freshly framed shards"
    for b in range(NBATCH):
        assert torch.equal(unframed[b, :, :S].reshape(nst, total, S), batch[b, :, :, :S]), "crc32block round trip differs"
    blk_bytes = nsh * (S + flen)  # read the payload and write the frames, or the reverse
    out.update({
        "crc32block_encode_data_GBps": rate(nsh * S, blk_enc_ms),
        "crc32block_encode_roofline_frac": frac(blk_bytes, blk_enc_ms),
        "crc32block_decode_data_GBps": rate(nsh * S, blk_dec_ms),
        "crc32block_decode_roofline_frac": frac(blk_bytes, blk_dec_ms),
        "secondary_note": ("each operation repeated for ~op_seconds of device time over the rotated batches, "
                           "HIP events on the launch stream; roofline fractions use the same algorithmic bytes"),
    })
    del framed, unframed
    # also against a measured device-copy peak -- torch's device-to-device copy of
    # one batch (716 MB) into a scratch batch, rotated like the step, 2 x bytes moved per copy
    scratch = torch.empty_like(batch[0])
    with torch.cuda.stream(stream):
        copy_ms = timed(lambda b: scratch.copy_(batch[b]))
    copy_bytes = 2 * batch[0].numel()
    out["device_copy_GBps"] = rate(copy_bytes, copy_ms)
    out["device_copy_note"] = ("torch copy_ of one rotated batch into a scratch batch (the HIP runtime D2D copy, "
                               "__amd_rocclr_copyBuffer), read + write bytes / time")
    # the measured streaming ceiling: a flat float4 non-temporal copy (cfsec_stream_copy, the form of
    # tools/rot_probe.hip), same bytes and rotation -- the roofline's second denominator
    from chubaofs_amd import _lib
    nb = batch[0].numel() // 16 * 16
    with torch.cuda.stream(stream):
        fcopy_ms = timed(lambda b: _lib.check(_lib.lib().cfsec_stream_copy(
            ctypes.c_void_p(scratch.data_ptr()), ctypes.c_void_p(batch[b].data_ptr()), nb, stream.cuda_stream)))
    out["stream_copy_GBps"] = rate(2 * nb, fcopy_ms)
    out["stream_copy_note"] = ("cfsec_stream_copy (flat 16-byte non-temporal grid-stride copy) of one rotated batch: "
                               "read + write bytes / time, the device's measured 1:1 streaming ceiling")
    del scratch
    return out


def host_path(args, torch, dev, world):
    """PCIe-inclusive rate of the drop-in path itself -- shards in host memory, CFSEC_MEM_HOST, what
    the cgo shim passes (go/cfsec) -- never `value`: EC12P4 Encode of 4 stripes of 64 MiB blobs per
    cfsec_ec_encode_batch call, from page-locked (cfsec_host_alloc, the resourcepool hook) and from
    pageable memory, on every rank at once.  Aggregate = all ranks' data / the slowest rank's time."""
    import numpy as np

    from chubaofs_amd import _lib, codemode as cm, ec
    K, M, S, nst, reps = K_DATA, M_PARITY, args.shard_size, 4, 5
    enc = ec.NewEncoder(ec.Config(CodeMode=cm.GetTactic(cm.EC12P4), EnableVerify=False), device=dev.index)
    seed = np.random.default_rng(7).integers(0, 256, S, dtype=np.uint8)
    out = {"workload": f"EC12P4 Encode, {nst} stripes of 64 MiB blobs (S={S}) per call, host memory, "
                       f"{reps} calls per rank, all ranks concurrently",
           "note": "PCIe-inclusive (H2D of 12 S + D2H of 4 S per stripe); the CPU baseline is the comparison"}
    for kind in ("pinned", "pageable"):
        buf = _lib.pinned_empty(nst * (K + M) * S) if kind == "pinned" else np.zeros(nst * (K + M) * S, np.uint8)
        stripes = [[buf[(s * (K + M) + i) * S:(s * (K + M) + i + 1) * S] for i in range(K + M)] for s in range(nst)]
        for s in range(nst):
            for i in range(K):
                stripes[s][i][:] = np.roll(seed, 977 * (s * K + i))
        assert enc.EncodeBatch(stripes) == [0] * nst
        assert enc.Verify(stripes[nst - 1])
        if world > 1:
            torch.distributed.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            st = enc.EncodeBatch(stripes)
        dt = time.perf_counter() - t0
        assert st == [0] * nst
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64, device=dev)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            dt = float(t.item())
        out[kind] = {"data_GBps": round(world * nst * K * S * reps / dt / 1e9, 2),
                     "pcie_GBps": round(world * nst * (K + M) * S * reps / dt / 1e9, 2),
                     "per_gpu_data_GBps": round(nst * K * S * reps / dt / 1e9, 2), "n_gpus": world}
        del stripes, buf
    # the link's measured peaks on this rank (page-locked <-> HBM copies of 256 MiB, each direction alone and
    # both at once on two streams): the path moves 12 S host-to-device and 4 S device-to-host per stripe, so
    # its host-to-device bytes (= data bytes) against the H2D peak is how close it runs to the PCIe roofline
    n = 256 << 20
    h_src = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    h_dst = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d_a = torch.empty(n, dtype=torch.uint8, device=dev)
    d_b = torch.empty(n, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def copies(h2d, d2h, reps=8):
        for _ in range(2):
            if h2d:
                with torch.cuda.stream(s1):
                    d_a.copy_(h_src, non_blocking=True)
            if d2h:
                with torch.cuda.stream(s2):
                    h_dst.copy_(d_b, non_blocking=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            if h2d:
                with torch.cuda.stream(s1):
                    d_a.copy_(h_src, non_blocking=True)
            if d2h:
                with torch.cuda.stream(s2):
                    h_dst.copy_(d_b, non_blocking=True)
        torch.cuda.synchronize()
        return reps * n / (time.perf_counter() - t0) / 1e9

    h2d, d2h = copies(True, False), copies(False, True)
    both = copies(True, True)
    out["pcie_peaks"] = {"h2d_GBps": round(h2d, 2), "d2h_GBps": round(d2h, 2),
                         "bidirectional_each_GBps": round(both, 2),
                         "note": "torch copies between page-locked host memory and HBM, 256 MiB, per rank"}
    for kind in ("pinned", "pageable"):
        out[kind]["h2d_frac_of_measured_peak"] = round(out[kind]["per_gpu_data_GBps"] / h2d, 3)
    del h_src, h_dst, d_a, d_b
    return out


# ----------------------------------------------------------------- BASELINE configs[4] over N GPUs
def multi_gpu_repair(args, torch, dev, rank, world):
    """BASELINE.json configs[4]: an EC16P20L2 repair tasklet (64 bids x S = 262,144, bad {0,1,16,17})
    whose shards are spread over the job's GPUs -- shard i of every bid on rank i % N -- repaired by
    chubaofs_amd/repair.py: all_to_all of every survivor's column slice over RCCL (xGMI), the
    reference's Reconstruct + Verify per bid on each rank's columns (blobnode/work_shard_recover.go:
    751-760), all_reduce of the per-bid status, all_to_all of the rebuilt slices back to their owners.
    Gate: the bad rows are zeroed in every rank's shards before the timed calls, and after them every
    rebuilt row equals the golden row, every bid's status is OK.  value = the tasklet's data bytes
    (16 * S * 64) per call / call time (barrier + sync both sides, max over ranks); at N = 1 the
    exchange is a local copy."""
    from chubaofs_amd import codemode as cm, ec, repair

    t5 = cm.GetTactic(cm.EC16P20L2)
    n, N5, nb, S = t5.N + t5.M + t5.L, t5.N, 64, 262144
    bad = [0, 1, 16, 17]
    enc = ec.NewEncoder(ec.Config(CodeMode=t5, EnableVerify=False), device=dev.index)
    # every rank builds the same tasklet (same seed) and keeps the shards it owns
    g = torch.Generator(device=dev)
    g.manual_seed(0xC5)
    full = torch.empty((nb, n, S), dtype=torch.uint8, device=dev)
    full[:, :N5] = torch.randint(0, 256, (nb, N5, S), generator=g, device=dev, dtype=torch.uint8)
    st = enc.EncodeBatchAsync([[full[b, i] for i in range(n)] for b in range(nb)])
    assert st == [0] * nb
    torch.cuda.synchronize()
    mine = repair.owned(rank, n, world)
    local = full[:, mine].contiguous()
    mine_bad = [e for e in bad if repair.owner(e, world) == rank]
    golden = full[:, mine_bad].clone()
    del full
    torch.cuda.empty_cache()
    for q, i in enumerate(mine):
        if i in bad:
            local[:, q].zero_()
    backend = torch.distributed.get_backend() if world > 1 else "none (world 1: local copies)"

    def call(timer=None, crcs=False):
        return repair.repair_batch(enc, local, bad, rank, world, crcs=crcs, timer=timer)

    for _ in range(2):
        call()
    torch.cuda.synchronize()
    steps = max(5, args.steps // 2)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    outs = [call() for _ in range(steps)]
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(tt, op=torch.distributed.ReduceOp.MAX)
        el = float(tt.item())
    # gate: every bid of every timed call verified OK (the fused pass recomputes all parities from the
    # rebuilt data rows and compares the 18 stored ones), and the rebuilt rows, written in place into
    # the zeroed rows of `local`, equal the golden rows
    for r in outs:
        assert r.status == [0] * nb, "C5 multi-GPU repair: a bid failed"
    assert outs[-1].index == mine_bad and torch.equal(outs[-1].rows, golden), "C5 multi-GPU repair: rebuilt rows differ"
    del outs
    # phase breakdown (HIP events on this rank's stream) and the checksummed form, averaged
    phases, reps = {}, 5
    for _ in range(reps):
        tm = {}
        call(timer=tm)
        for k_, v in tm.items():
            phases[k_] = phases.get(k_, 0.0) + v / reps
    tc0 = time.perf_counter()
    rc = None
    for _ in range(reps):
        rc = call(crcs=True)
    torch.cuda.synchronize()
    crc_ms = (time.perf_counter() - tc0) / reps * 1e3
    gh = golden.cpu().numpy()
    import zlib
    for q in range(len(mine_bad)):
        for b in (0, nb - 1):
            assert int(rc.crcs[b, q]) == zlib.crc32(gh[b, q].tobytes()) & 0xFFFFFFFF, "C5 multi-GPU checksum"
    st_ = rc.stats
    data = N5 * S * nb
    ph = {k_: torch.tensor([v], dtype=torch.float64, device=dev) for k_, v in phases.items()}
    if world > 1:
        for v in ph.values():
            torch.distributed.all_reduce(v, op=torch.distributed.ReduceOp.MAX)
    ph = {k_: round(float(v.item()), 4) for k_, v in ph.items()}
    xbytes = st_.get("exchange_bytes_received", 0)
    return {
        "workload": (f"EC16P20L2 repair tasklet, {nb} bids x S={S}, bad {{0,1,16,17}}, shard i of every bid on "
                     f"rank i % {world}; column-split Reconstruct + Verify per bid (repair.py 'columns')"),
        "world": world, "backend": backend,
        "data_GBps": round(data * steps / el / 1e9, 2),
        "ms_per_tasklet": round(el / steps * 1e3, 4),
        "phases_ms_max_over_ranks": ph,
        "exchange_bytes_received_per_rank": xbytes,
        "exchange_bytes_sent_per_rank": st_.get("exchange_bytes_sent", 0),
        "return_bytes_received_per_rank": st_.get("return_bytes_received", 0),
        "exchange_GBps_per_rank": round(xbytes / (ph["exchange_ms"] * 1e-3) / 1e9, 2) if ph.get("exchange_ms") else None,
        "rows_shipped_per_bid": st_.get("rows_shipped"), "columns_per_rank": st_.get("columns"),
        "with_crc_ms_per_tasklet": round(crc_ms, 4),
        "timing": ("data_GBps: tasklets back to back, barrier + sync both sides, max over ranks; phases: HIP events "
                   "around the forward exchange, the decode and the return exchange + status reduction (mean of "
                   f"{reps}, max over ranks); with_crc: the call returning the rebuilt shards' checksums (zlib-checked)"),
        "gate": ("bad rows zeroed before the timed calls; every bid of every call verified OK; the rebuilt rows "
                 "(in place in each rank's shards) equal the golden rows afterwards"),
    }


# ----------------------------------------------------------------- segment ReconstructData latency
def segment_latency(args, torch, dev, cpu):
    """access's degraded read of a byte range (access/stream_get.go:420-427): ReconstructData over
    every shard's segment [off, off + seg) of a blob with two data shards bad, one call per read --
    a latency path.  Per-call wall time (median of repeated calls) for segments in pageable host
    memory (what a Go caller has), page-locked host memory (cfsec_host_alloc) and HBM, with the
    klauspost-strategy CPU port on the same segment (4 threads as the reference with GFNI, and 1).
    `gpu_wins_from_bytes` per mode: the smallest measured segment size at which the GPU call beats
    the CPU port -- below it a caller should decode on the CPU."""
    import numpy as np

    from chubaofs_amd import _lib, codemode as cm, ec
    out = {"workload": ("ReconstructData of one segment per shard at offset 4096 inside a 64 MiB blob, bad data "
                        "shards {0, 1}; median of repeated calls"), "modes": {}}
    reps = 40
    if cpu:
        from oracle import oracle as O

    def med(fn, n=reps):
        fn()
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        ts.sort()
        return ts[len(ts) // 2] * 1e6

    for name, mode in (("EC6P6", cm.EC6P6), ("EC12P4", cm.EC12P4)):
        t = cm.GetTactic(mode)
        N, n = t.N, t.N + t.M
        enc = ec.NewEncoder(ec.Config(CodeMode=t, EnableVerify=False), device=dev.index)
        rows = {}
        for seg in (4096, 65536, 1 << 20):
            off = 4096
            S = off + seg
            rng = np.random.default_rng(seg + N)
            full = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(N)] + [np.zeros(S, np.uint8) for _ in range(t.M)]
            enc.Encode(full)
            gold = [x[off:off + seg].copy() for x in full]
            bad = [0, 1]
            r = {}
            pin = _lib.pinned_empty(n * seg)
            pinned = [pin[i * seg:(i + 1) * seg] for i in range(n)]
            devt = [torch.from_numpy(g.copy()).to(dev) for g in gold]
            for kind in ("pageable", "pinned", "device"):
                if kind == "pageable":
                    segs = [x[off:off + seg] for x in full]
                elif kind == "pinned":
                    for i in range(n):
                        pinned[i][:] = gold[i]
                    segs = list(pinned)
                else:
                    segs = list(devt)

                def call():
                    v = list(segs)
                    enc.ReconstructData(v, bad)
                    if kind == "device":
                        torch.cuda.synchronize()

                r[kind + "_us"] = round(med(call), 1)
                # the C ABI alone, as cgo calls it: the shard vector marshalled once, no torch
                # synchronize -- the Python layer's Marshal and ctypes costs ~25-35 us of the figure
                # above (tools/r5_latency.py).  HBM shards on a stream of their own (the call is
                # synchronous); host shards with a NULL stream, as the Go shim passes them
                # (CFSEC_MEM_HOST: page-locked rows read and written by the kernel over PCIe,
                # pageable rows staged through HBM).
                from chubaofs_amd._shards import Marshal
                m = Marshal(list(segs))
                badarr = (ctypes.c_int * 2)(*bad)
                own = torch.cuda.Stream(dev)
                torch.cuda.synchronize()
                cst = own.cuda_stream if kind == "device" else None

                def cabi():
                    _lib.check(enc._L.cfsec_ec_reconstruct_data(enc._h, m.ptr(), m.n, badarr, 2, m.mem, cst))

                r[kind + "_cabi_us"] = round(med(cabi), 1)
                got = [np.asarray(x.cpu().numpy() if kind == "device" else x) for x in segs[:N]]
                assert all(np.array_equal(got[i], gold[i]) for i in range(N)), f"segment {name} {seg} {kind}"
            if cpu:
                G = O.build_matrix(N, n)
                valid = [i for i in range(n) if i not in bad][:N]
                err, dec = O.invert(G[valid])
                assert err == 0
                ins = [gold[i] for i in valid]
                outs = [np.zeros(seg, np.uint8) for _ in bad]
                for thr in (4, 1):
                    r[f"cpu_port_{thr}t_us"] = round(med(lambda: O.simd_code(dec[bad], ins, outs, thr)), 1)
                assert all(np.array_equal(outs[j], gold[b]) for j, b in enumerate(bad))
            rows[str(seg)] = r
            del pin, pinned, devt
        wins = {}
        if cpu:
            for kind in ("pageable", "pinned", "device", "pageable_cabi", "pinned_cabi", "device_cabi"):
                w = [int(s) for s, r in rows.items()
                     if r[kind + "_us"] < min(r["cpu_port_4t_us"], r["cpu_port_1t_us"])]
                wins[kind] = min(w) if w else None
        out["modes"][name] = {"by_segment_bytes": rows, "gpu_wins_from_bytes": wins}
    out["note"] = ("gpu_wins_from_bytes: smallest measured segment where the GPU call (wall, incl. staging and "
                   "sync) beats the faster of the CPU port's 1- and 4-thread calls; None: the CPU port wins at every "
                   "measured size.  *_us: through the Python ec.Encoder (Marshal + ctypes + torch synchronize); "
                   "*_cabi_us: the C ABI call alone (what the Go shim's cgo call costs): HBM shards synchronous on a "
                   "stream of their own, host shards (pageable, or page-locked by cfsec_host_alloc) with a NULL stream "
                   "as the shim passes")
    return out


# ----------------------------------------------------------------- BASELINE configs 1, 4, 5
def cpu_rate(fn, seconds):
    """Calls of fn per second over ~seconds (after one warm call)."""
    fn()
    n, t0 = 0, time.perf_counter()
    while True:
        fn()
        n += 1
        dt = time.perf_counter() - t0
        if dt >= seconds:
            return n / dt


def cpu_saturated_rate(make_worker, seconds, callers):
    """BASELINE.md's saturated CPU mode for a config: `callers` concurrent single-threaded callers
    (one per usable host CPU), each with its own buffers (make_worker(w) returns its call); total
    calls per second."""
    import threading
    callers = max(1, int(callers))
    fns = [make_worker(w) for w in range(callers)]
    for f in fns:
        f()
    done = [0] * callers
    stop = time.perf_counter() + seconds

    def loop(w):
        while time.perf_counter() < stop:
            fns[w]()
            done[w] += 1

    t0 = time.perf_counter()
    th = [threading.Thread(target=loop, args=(w,)) for w in range(callers)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    return sum(done) / (time.perf_counter() - t0)


def gated_calls(torch, stream, call, nbatch, seconds, zero, check, sync_call):
    """Time a config's GPU calls with the headline's gate: after two warm calls per batch the rows
    the calls write are zeroed (`zero`), the timed calls run over the rotated batches (at least one
    per batch), and afterwards every written row must equal the golden bytes again (`check`).

    sync_call: the calls are synchronous library calls -> calls per second of wall time.  Else they
    are enqueued on `stream`: each call is bracketed by its own HIP event pair on that stream, so the
    sum of the pairs is the device time of the calls' kernels alone ("kernel-only"), and the first
    to last event the pipelined rate (host planning of call i+1 overlapping the kernels of call i).
    Returns dict(calls_per_s=..., kernel_ms_per_call=..., n=...)."""
    # Whatever the caller prepared on other streams (torch's copies onto its current stream, e.g. the
    # scattered C5 pool) is complete before the first call: the asynchronous calls run on `stream`,
    # which does not wait for torch's stream.  Without this the scattered C5 run's first warm calls
    # could read half-copied rows under load -- the "false Verify" flags of the N = 2 rehearsals in
    # rounds 4 and 5 (flags set by those warm calls, never cleared; the rows right at the end).
    torch.cuda.synchronize()
    for i in range(2 * nbatch):
        call(i)
    torch.cuda.synchronize()
    zero()
    torch.cuda.synchronize()
    if sync_call:
        n, t0 = 0, time.perf_counter()
        while True:
            call(n)
            n += 1
            dt = time.perf_counter() - t0
            if dt >= seconds and n >= nbatch:
                break
        torch.cuda.synchronize()
        check()
        return {"calls_per_s": n / dt, "n": n}
    # estimate the count from a short untimed run, then the timed run with per-call events
    t0 = time.perf_counter()
    for i in range(nbatch):
        call(i)
    torch.cuda.synchronize()
    est = max((time.perf_counter() - t0) / nbatch, 1e-5)
    n = max(3 * nbatch, int(seconds / est) // nbatch * nbatch)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for i in range(n):
        evs[i][0].record(stream)
        call(i)
        evs[i][1].record(stream)
    torch.cuda.synchronize()
    check()
    kern = sum(a.elapsed_time(b) for a, b in evs) / n
    wall = evs[0][0].elapsed_time(evs[-1][1]) / n
    return {"calls_per_s": 1e3 / wall, "kernel_ms_per_call": kern, "n": n}


def other_configs(args, torch, dev, stream, cpu):
    """BASELINE.json configs[0], [3] and [4] on this GPU, each with the klauspost-strategy CPU port
    (oracle/cpu_simd.c) timed beside it on the same shapes: 4 threads per call as the reference with
    GFNI, and saturated (one single-threaded caller per usable host CPU).  Every GPU rate is gated
    like the headline (gated_calls: the rows the timed calls write are zeroed first and must equal the
    golden bytes afterwards, so a kernel that writes nothing fails).  C4 / C5 report both the
    synchronous batch calls a caller makes (planning, launches, sync) and the asynchronous calls
    (cfsec_ec_*_batch_async) on one stream, with their kernel-only time from per-call HIP events."""
    import zlib

    import numpy as np

    from chubaofs_amd import _lib, codemode as cm, ec, reedsolomon
    from chubaofs_amd._shards import BatchMarshal

    out = {}
    secs = max(0.3, args.op_seconds)
    cpu_secs = max(1.0, args.cpu_seconds / 5)
    if cpu:
        from oracle import oracle as O
    gfni = cpu and O.simd_features()["gfni"]
    thr = 4 if gfni else 8
    callers = host_cpu_share()["usable"]
    frac = lambda nbytes, ms: round(nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)

    # ---- C1: EC6P6 encode of 1 MiB blobs, 256 blobs per batch (configs[0])
    k, m, nb = 6, 6, 256
    S1 = (1 << 20) + k - 1
    S1 //= k  # 174,763
    p1 = (S1 + 255) // 256 * 256
    b1 = torch.randint(0, 256, (NBATCH, nb, k + m, p1), dtype=torch.uint8, device=dev)
    r6 = reedsolomon.New(k, m, device=dev.index)
    pt = [(ctypes.c_void_p * (nb * (k + m)))(*[b1[b].data_ptr() + (s * (k + m) + i) * p1 for s in range(nb)
                                              for i in range(k + m)]) for b in range(NBATCH)]
    for b in range(NBATCH):
        r6.encode_batch(pt[b], S1, nb, stream=stream)
    torch.cuda.synchronize()
    gold1 = b1[:, :, k:, :S1].clone()

    def check1():
        assert torch.equal(b1[:, :, k:, :S1], gold1), "C1: parity after the timed encodes differs from the golden"

    r = gated_calls(torch, stream, lambda i: r6.encode_batch(pt[i % NBATCH], S1, nb, stream=stream), NBATCH, secs,
                    lambda: b1[:, :, k:, :].zero_(), check1, sync_call=False)
    ms = r["kernel_ms_per_call"]
    c1 = {"workload": f"EC6P6 encode, {nb} blobs of 1 MiB (S={S1}), device-resident, one launch",
          "data_GBps": round(k * S1 * nb / (ms * 1e-3) / 1e9, 1),
          "roofline_frac": frac((k + m) * S1 * nb, ms),
          "avg_launch_ms": round(ms, 4), "algorithmic_bytes_per_launch": (k + m) * S1 * nb,
          "gate": "parity rows zeroed before the timed launches, equal to the golden parity after"}
    # access's Put checksums every shard right after Encode (stream_put.go:249-253): the same batches
    # through cfsec_rs_encode_crc_batch, all 12 checksums per blob (zlib-checked)
    cw1 = torch.zeros((NBATCH, nb * (k + m)), dtype=torch.int32, device=dev)
    rc = gated_calls(torch, stream, lambda i: r6.encode_crc_batch(pt[i % NBATCH], S1, nb, cw1[i % NBATCH].data_ptr(),
                                                                   stream=stream),
                     NBATCH, secs, lambda: b1[:, :, k:, :].zero_(), check1, sync_call=False)
    w1h = cw1[0].cpu().numpy().view(np.uint32).reshape(nb, k + m)
    g1h = b1[0, :, :, :S1].cpu().numpy()
    for s_ in (0, nb - 1):
        for i in range(k + m):
            assert int(w1h[s_, i]) == zlib.crc32(g1h[s_, i].tobytes()) & 0xFFFFFFFF, f"C1 checksum {s_} {i}"
    c1.update({"encode_crc_kernel_ms": round(rc["kernel_ms_per_call"], 4),
               "encode_crc_roofline_frac": frac((k + m) * S1 * nb, rc["kernel_ms_per_call"]),
               "encode_crc_over_encode": round(rc["kernel_ms_per_call"] / ms, 3)})
    del cw1
    if cpu:
        full = O.build_matrix(k, k + m)
        h = b1[0, 0, :k, :S1].cpu().numpy()
        data = [np.ascontiguousarray(h[i]) for i in range(k)]
        par = [np.zeros(S1, np.uint8) for _ in range(m)]
        rate = cpu_rate(lambda: O.simd_code(full[k:], data, par, thr), cpu_secs)
        ok = all(np.array_equal(par[r_], b1[0, 0, k + r_, :S1].cpu().numpy()) for r_ in range(m))

        def w1(w):
            d = [np.roll(x, w) for x in data]
            p = [np.zeros(S1, np.uint8) for _ in range(m)]
            return lambda: O.simd_code(full[k:], d, p, 1)

        sat = cpu_saturated_rate(w1, cpu_secs, callers)
        c1["cpu_baseline"] = {"value": round(k * S1 * rate / 1e9, 3), "unit": "GB/s", "cores": thr, "kind": "port",
                              "sample": f"one 1 MiB blob encoded repeatedly for ~{cpu_secs:.0f}s",
                              "parity_equals_gpu": bool(ok),
                              "saturated": {"value": round(k * S1 * sat / 1e9, 3), "unit": "GB/s", "cores": callers,
                                            "sample": f"{callers} single-threaded callers, one blob each"}}
    out["C1_EC6P6_1MiB_encode"] = c1
    del b1, pt, gold1

    # ---- C4: EC6P10L2 fused LRC encode + AZ-local repair, 4 MiB blobs (configs[3])
    t4 = cm.GetTactic(cm.EC6P10L2)
    N, M, L = t4.N, t4.M, t4.L
    tot4 = N + M + L
    S4 = ((4 << 20) + N - 1) // N  # 699,051
    p4 = (S4 + 255) // 256 * 256
    nb4 = 48
    e4 = ec.NewEncoder(ec.Config(CodeMode=t4, EnableVerify=False), device=dev.index)
    b4 = torch.randint(0, 256, (NBATCH, nb4, tot4, p4), dtype=torch.uint8, device=dev)
    bms = [BatchMarshal([[b4[b, s, i, :S4] for i in range(tot4)] for s in range(nb4)], tot4) for b in range(NBATCH)]
    st4 = (ctypes.c_int * nb4)()
    for b in range(NBATCH):
        _lib.check(e4._L.cfsec_ec_encode_batch(e4._h, bms[b].arr, tot4, nb4, bms[b].mem, st4))
    torch.cuda.synchronize()
    gold4 = b4[:, :, :, :S4].clone()

    def check4(rows):
        def f():
            assert torch.equal(b4[:, :, rows, :S4], gold4[:, :, rows]), f"C4: rows {rows} differ from the golden"
        return f

    def zero4(rows):
        return lambda: b4[:, :, rows, :].zero_()

    par4 = list(range(N, tot4))

    def enc4(i):
        bm = bms[i % NBATCH]
        _lib.check(e4._L.cfsec_ec_encode_batch(e4._h, bm.arr, tot4, nb4, bm.mem, st4))

    def enc4a(i):
        bm = bms[i % NBATCH]
        _lib.check(e4._L.cfsec_ec_encode_batch_async(e4._h, bm.arr, tot4, nb4, st4, None, None, stream.cuda_stream))

    rs = gated_calls(torch, stream, enc4, NBATCH, secs, zero4(par4), check4(par4), sync_call=True)
    assert list(st4) == [0] * nb4
    ra = gated_calls(torch, stream, enc4a, NBATCH, secs, zero4(par4), check4(par4), sync_call=False)
    assert list(st4) == [0] * nb4
    # access's Put checksums every shard of the encoded blob (stream_put.go:249-253): the same calls
    # returning all 18 checksums per blob
    cw4 = torch.zeros((NBATCH, nb4 * tot4), dtype=torch.int32, device=dev)

    def enc4c(i):
        bm = bms[i % NBATCH]
        _lib.check(e4._L.cfsec_ec_encode_batch_async(e4._h, bm.arr, tot4, nb4, st4, None,
                                                     ctypes.c_void_p(cw4[i % NBATCH].data_ptr()), stream.cuda_stream))

    rc4 = gated_calls(torch, stream, enc4c, NBATCH, secs, zero4(par4), check4(par4), sync_call=False)
    assert list(st4) == [0] * nb4
    w4 = cw4[0].cpu().numpy().view(np.uint32).reshape(nb4, tot4)
    g4h = gold4[0].cpu().numpy()
    for s_ in (0, nb4 - 1):
        for i in range(tot4):
            assert int(w4[s_, i]) == zlib.crc32(g4h[s_, i].tobytes()) & 0xFFFFFFFF, f"C4 checksum {s_} {i}"
    enc_bytes = tot4 * S4 * nb4
    c4 = {"workload": f"EC6P10L2 fused LRC encode (global + 2 local parities in one pass), {nb4} blobs of 4 MiB (S={S4})",
          "encode_data_GBps": round(N * S4 * nb4 * rs["calls_per_s"] / 1e9, 1),
          "encode_roofline_frac": round(enc_bytes * rs["calls_per_s"] / 1e9 / HBM_PEAK_GBPS, 4),
          "encode_async_data_GBps": round(N * S4 * nb4 * ra["calls_per_s"] / 1e9, 1),
          "encode_kernel_ms": round(ra["kernel_ms_per_call"], 4),
          "encode_kernel_roofline_frac": frac(enc_bytes, ra["kernel_ms_per_call"]),
          "encode_crc_kernel_ms": round(rc4["kernel_ms_per_call"], 4),
          "encode_crc_kernel_roofline_frac": frac(enc_bytes, rc4["kernel_ms_per_call"]),
          "encode_crc_over_kernel": round(rc4["kernel_ms_per_call"] / ra["kernel_ms_per_call"], 3)}
    # AZ-local repair: AZ0's local stripe (8 + 1 shards) per blob, local index 0 lost
    idx0, _, _ = t4.LocalStripeInAZ(0)
    lsz = len(idx0)
    lbm = [BatchMarshal([[b4[b, s, i, :S4] for i in idx0] for s in range(nb4)], lsz) for b in range(NBATCH)]
    bad = (ctypes.c_int * nb4)(*([0] * nb4))
    off = (ctypes.c_int * (nb4 + 1))(*range(nb4 + 1))
    fl4 = torch.zeros(nb4, dtype=torch.int32, device=dev)

    def rep4(i):
        bm = lbm[i % NBATCH]
        _lib.check(e4._L.cfsec_ec_reconstruct_batch(e4._h, bm.arr, lsz, nb4, bad, off, 1, bm.mem, st4))

    def rep4a(i):
        bm = lbm[i % NBATCH]
        _lib.check(e4._L.cfsec_ec_reconstruct_batch_async(e4._h, bm.arr, lsz, nb4, bad, off, 1, st4,
                                                          fl4.data_ptr(), None, stream.cuda_stream))

    lost = [idx0[0]]
    rs = gated_calls(torch, stream, rep4, NBATCH, secs, zero4(lost), check4(lost), sync_call=True)
    assert list(st4) == [0] * nb4
    ra = gated_calls(torch, stream, rep4a, NBATCH, secs, zero4(lost), check4(lost), sync_call=False)
    assert list(st4) == [0] * nb4 and not bool(fl4.any().item()), "C4: local Verify failed"
    rep_bytes = lsz * S4 * nb4
    c4.update({"local_repair_data_GBps": round((lsz - 1) * S4 * nb4 * rs["calls_per_s"] / 1e9, 1),
               "local_repair_roofline_frac": round(rep_bytes * rs["calls_per_s"] / 1e9 / HBM_PEAK_GBPS, 4),
               "local_repair_async_data_GBps": round((lsz - 1) * S4 * nb4 * ra["calls_per_s"] / 1e9, 1),
               "local_repair_kernel_ms": round(ra["kernel_ms_per_call"], 4),
               "local_repair_kernel_roofline_frac": frac(rep_bytes, ra["kernel_ms_per_call"]),
               "timing": ("*_data_GBps / *_roofline_frac: synchronous batch calls on device memory (planning + "
                          "launch + sync); *_async_*: cfsec_ec_*_batch_async back to back on one stream; "
                          "*_kernel_*: per-call HIP event pairs around the async calls (device time only)"),
               "gate": "rows each timed call writes zeroed before, equal to the golden after (sync and async runs)"})
    # the floor under any synchronous call: one trivial kernel launched and waited for (HIP launch +
    # completion latency), the part of a synchronous call's time no host-side planning cache removes
    tiny = torch.zeros(64, dtype=torch.int32, device=dev)
    fl = []
    for _ in range(200):
        t0 = time.perf_counter()
        tiny.add_(1)
        torch.cuda.synchronize()
        fl.append(time.perf_counter() - t0)
    fl.sort()
    c4["sync_floor_us"] = round(fl[len(fl) // 2] * 1e6, 1)
    c4["local_repair_sync_call_us"] = round(1e6 / rs["calls_per_s"], 1)
    if cpu:
        G = O.build_matrix(N, N + M)
        Lm = O.build_matrix(lsz - 1, lsz)
        h = b4[0, 0, :, :S4].cpu().numpy()
        data = [np.ascontiguousarray(h[i]) for i in range(N)]
        gpar = [np.zeros(S4, np.uint8) for _ in range(M)]
        lpar = [np.zeros(S4, np.uint8) for _ in range(L)]

        def cpu_enc4(data, gpar, lpar, thr):  # lrcencoder.go:35-82: global Encode, then each AZ's local Encode
            def f():
                O.simd_code(G[N:], data, gpar, thr)
                full = data + gpar
                for a in range(t4.AZCount):
                    ia, _, _ = t4.LocalStripeInAZ(a)
                    O.simd_code(Lm[lsz - 1:], [full[i] for i in ia[:lsz - 1]], [lpar[a]], thr)
            return f

        rate_c = cpu_rate(cpu_enc4(data, gpar, lpar, thr), cpu_secs)
        ok = all(np.array_equal(gpar[r_], h[N + r_]) for r_ in range(M)) and \
            all(np.array_equal(lpar[a], h[N + M + a]) for a in range(L))
        sat_e = cpu_saturated_rate(lambda w: cpu_enc4([x.copy() for x in data], [np.zeros(S4, np.uint8) for _ in range(M)],
                                                      [np.zeros(S4, np.uint8) for _ in range(L)], 1),
                                   cpu_secs, callers)
        err, dec = O.invert(Lm[1:lsz])  # local stripe with index 0 lost: survivors 1..8
        assert err == 0
        surv = [np.ascontiguousarray(h[i]) for i in idx0[1:]]
        rebuilt = [np.zeros(S4, np.uint8)]
        rate_cr = cpu_rate(lambda: O.simd_code(dec[:1], surv, rebuilt, thr), cpu_secs)

        def w4r(w):
            sv = [x.copy() for x in surv]
            rb = [np.zeros(S4, np.uint8)]
            return lambda: O.simd_code(dec[:1], sv, rb, 1)

        sat_r = cpu_saturated_rate(w4r, cpu_secs, callers)
        c4["cpu_baseline"] = {
            "encode": {"value": round(N * S4 * rate_c / 1e9, 3), "unit": "GB/s", "cores": thr, "kind": "port",
                       "sample": "one blob: global (6,10) encode + two local (8,1) encodes, repeated",
                       "parity_equals_gpu": bool(ok),
                       "saturated": {"value": round(N * S4 * sat_e / 1e9, 3), "unit": "GB/s", "cores": callers}},
            "local_repair": {"value": round((lsz - 1) * S4 * rate_cr / 1e9, 3), "unit": "GB/s", "cores": thr,
                             "kind": "port", "sample": "one local stripe: the lost shard rebuilt from 8, repeated",
                             "equals_original": bool(np.array_equal(rebuilt[0], h[idx0[0]])),
                             "saturated": {"value": round((lsz - 1) * S4 * sat_r / 1e9, 3), "unit": "GB/s",
                                           "cores": callers}}}
    out["C4_EC6P10L2_lrc_encode_local_repair"] = c4
    del bms, lbm, b4, gold4

    # ---- C5: EC16P20L2 repair tasklet, 64 bids of 4 MiB blobs, erased {0, 1, 16, 17} (configs[4]),
    # on one GPU: Reconstruct + Verify per bid (blobnode/work_shard_recover.go:751-757)
    t5 = cm.GetTactic(cm.EC16P20L2)
    N5, tot5 = t5.N, t5.N + t5.M + t5.L
    S5 = max(((4 << 20) + N5 - 1) // N5, t5.MinShardSize)  # 262,144
    p5 = (S5 + 255) // 256 * 256
    nb5 = 64
    e5 = ec.NewEncoder(ec.Config(CodeMode=t5, EnableVerify=False), device=dev.index)
    b5 = torch.randint(0, 256, (NBATCH, nb5, tot5, p5), dtype=torch.uint8, device=dev)
    bm5 = [BatchMarshal([[b5[b, s, i, :S5] for i in range(tot5)] for s in range(nb5)], tot5) for b in range(NBATCH)]
    st5 = (ctypes.c_int * nb5)()
    for b in range(NBATCH):
        _lib.check(e5._L.cfsec_ec_encode_batch(e5._h, bm5[b].arr, tot5, nb5, bm5[b].mem, st5))
    torch.cuda.synchronize()
    gold5 = b5[:, :, :, :S5].clone()
    er5 = [0, 1, 16, 17]
    bad5 = (ctypes.c_int * (4 * nb5))(*(er5 * nb5))
    off5 = (ctypes.c_int * (nb5 + 1))(*range(0, 4 * nb5 + 1, 4))
    fl5 = torch.zeros(nb5, dtype=torch.int32, device=dev)

    def check5():
        assert torch.equal(b5[:, :, er5, :S5], gold5[:, :, er5]), "C5: rebuilt rows differ from the golden"

    def rep5(i):
        bm = bm5[i % NBATCH]
        _lib.check(e5._L.cfsec_ec_reconstruct_batch(e5._h, bm.arr, tot5, nb5, bad5, off5, 1, bm.mem, st5))

    def rep5a(i):
        bm = bm5[i % NBATCH]
        _lib.check(e5._L.cfsec_ec_reconstruct_batch_async(e5._h, bm.arr, tot5, nb5, bad5, off5, 1, st5,
                                                          fl5.data_ptr(), None, stream.cuda_stream))

    # the same tasklet returning the rebuilt shards' checksums (blobnode's ShardCrc32 of each repaired
    # shard, work_shard_recover.go:335-342): device words [bid][shard], written on the stream
    cw5 = torch.zeros((NBATCH, nb5 * tot5), dtype=torch.int32, device=dev)

    def rep5c(i):
        bm = bm5[i % NBATCH]
        _lib.check(e5._L.cfsec_ec_reconstruct_batch_async(e5._h, bm.arr, tot5, nb5, bad5, off5, 1, st5,
                                                          fl5.data_ptr(), ctypes.c_void_p(cw5[i % NBATCH].data_ptr()),
                                                          stream.cuda_stream))

    zero5 = lambda: b5[:, :, er5, :].zero_()

    def check5_status(what):
        """every bid's planning status OK and no Verify flag set -- else which bids, with the raw flag
        words (a CFSEC_BS_DEBUG_FLAGS=1 library writes 0x80000000 | compared row << 24 | column tile)"""
        fl = fl5.cpu().numpy().view(np.uint32)
        bad_st = {b: int(v) for b, v in enumerate(st5) if v}
        bad_fl = {b: hex(int(v)) for b, v in enumerate(fl) if v}
        assert not bad_st and not bad_fl, f"C5: Verify failed ({what}): status {bad_st} flags {bad_fl}"
    rs = gated_calls(torch, stream, rep5, NBATCH, secs, zero5, check5, sync_call=True)
    assert list(st5) == [0] * nb5
    ra = gated_calls(torch, stream, rep5a, NBATCH, secs, zero5, check5, sync_call=False)
    check5_status("async run")
    rc = gated_calls(torch, stream, rep5c, NBATCH, secs, zero5, check5, sync_call=False)
    check5_status("crc run")
    # the words against zlib on the golden rebuilt rows (every bid of batch 0), 0 for the others
    w5 = cw5[0].cpu().numpy().view(np.uint32).reshape(nb5, tot5)
    g5h = gold5[0].cpu().numpy()
    for bid in range(nb5):
        for i in range(tot5):
            want = zlib.crc32(g5h[bid, i].tobytes()) & 0xFFFFFFFF if i in er5 else 0
            assert int(w5[bid, i]) == want, f"C5 checksum of bid {bid} shard {i}"
    # blobnode's own layout: every shard of the tasklet at its own address (a bid assembled from
    # per-vuid ShardsBuf buffers, work_shard_recover.go:711-716) -- the same rows copied into shuffled
    # slots of a pool, so no two rows share a stride
    rnd5 = np.random.default_rng(5)
    slot5 = p5 + 4096
    pool5 = torch.empty((NBATCH, nb5 * tot5 * slot5 + 4096), dtype=torch.uint8, device=dev)
    sc5, scv5 = [], []
    for b in range(NBATCH):
        perm = rnd5.permutation(nb5 * tot5)
        rows = [[None] * tot5 for _ in range(nb5)]
        for bid in range(nb5):
            for i in range(tot5):
                o = int(perm[bid * tot5 + i]) * slot5 + 256 * int(rnd5.integers(16))
                rows[bid][i] = pool5[b, o:o + S5]
                rows[bid][i].copy_(gold5[b, bid, i])
        scv5.append(rows)
        sc5.append(BatchMarshal(rows, tot5))

    def rep5s(i):
        bm = sc5[i % NBATCH]
        _lib.check(e5._L.cfsec_ec_reconstruct_batch_async(e5._h, bm.arr, tot5, nb5, bad5, off5, 1, st5,
                                                          fl5.data_ptr(), None, stream.cuda_stream))

    def zero5s():
        for rows in scv5:
            for bid in range(nb5):
                for i in er5:
                    rows[bid][i].zero_()

    def check5s():
        for b in range(NBATCH):
            got = torch.stack([torch.stack([scv5[b][bid][i] for i in er5]) for bid in range(nb5)])
            assert torch.equal(got, gold5[b, :, er5]), "C5 scattered: rebuilt rows differ from the golden"

    fl5.zero_()  # this run's flags only
    rsc = gated_calls(torch, stream, rep5s, NBATCH, secs, zero5s, check5s, sync_call=False)
    check5_status("scattered run")
    del sc5, scv5, pool5
    # per bid, one pass: reads 16 inputs + the 16 other global parities and the 2 local parities
    # it checks, writes 2 data + 2 parity rows (the local Verify rides in the global pass: the
    # separate AZ-local pass would re-read 2 x 19 shards)
    alg5 = (16 + 16 + 2 + 4) * S5
    c5 = {"workload": (f"EC16P20L2 repair tasklet on one GPU: {nb5} bids x S={S5}, erased {{0,1,16,17}}, "
                       "Reconstruct + Verify per bid in one cfsec_ec_reconstruct_batch: one fused pass per bid (bit-sliced "
                       "repair kernel; global and local parities checked in it)"),
          "data_GBps": round(N5 * S5 * nb5 * rs["calls_per_s"] / 1e9, 1),
          "roofline_frac": round(alg5 * nb5 * rs["calls_per_s"] / 1e9 / HBM_PEAK_GBPS, 4),
          "async_data_GBps": round(N5 * S5 * nb5 * ra["calls_per_s"] / 1e9, 1),
          "kernel_ms": round(ra["kernel_ms_per_call"], 4),
          "kernel_roofline_frac": frac(alg5 * nb5, ra["kernel_ms_per_call"]),
          "with_crc_kernel_ms": round(rc["kernel_ms_per_call"], 4),
          "scattered_kernel_ms": round(rsc["kernel_ms_per_call"], 4),
          "scattered_kernel_roofline_frac": frac(alg5 * nb5, rsc["kernel_ms_per_call"]),
          "scattered_note": ("the same tasklet with every shard at its own address (blobnode's per-vuid buffers): "
                             "cfsec_ec_reconstruct_batch_async device time per call, rebuilt rows checked against the "
                             "golden"),
          "with_crc_over_kernel": round(rc["kernel_ms_per_call"] / ra["kernel_ms_per_call"], 3),
          "with_crc_note": ("cfsec_ec_reconstruct_batch_async with the rebuilt shards' checksums (256 words per "
                            "call, checked against zlib on the golden rows): device time per call, and its ratio "
                            "to the call without checksums"),
          "algorithmic_bytes_per_bid": alg5,
          "timing": ("data_GBps / roofline_frac: synchronous cfsec_ec_reconstruct_batch calls (planning + launches + "
                     "sync); async_*: cfsec_ec_reconstruct_batch_async back to back on one stream; kernel_*: per-call "
                     "HIP event pairs around the async calls"),
          "gate": "rows {0,1,16,17} zeroed before the timed calls, equal to the golden after (sync and async runs)",
          "multi_gpu_note": "the same tasklet with its shards spread over the job's GPUs: C5_multi_gpu_repair"}
    if cpu:
        G5 = O.build_matrix(N5, N5 + t5.M)
        l5 = (N5 + t5.M) // t5.AZCount
        Lm5 = O.build_matrix(l5, l5 + 1)
        h = b5[0, 0, :, :S5].cpu().numpy()
        valid = [i for i in range(N5 + t5.M) if i not in er5][:N5]
        err, dec = O.invert(G5[valid])
        assert err == 0
        rows_data = dec[[0, 1]]
        prow = G5[[16, 17]]

        def cpu_rep5(sh, thr):  # Reconstruct (data rows, then parity rows) + Verify (global, then local)
            outs = [np.zeros(S5, np.uint8) for _ in range(4)]
            tmp = [np.zeros(S5, np.uint8) for _ in range(t5.M)]
            ltmp = [np.zeros(S5, np.uint8)]

            def f():
                ins = [sh[i] for i in valid]
                O.simd_code(rows_data, ins, outs[:2], thr)
                O.simd_code(prow, [sh[i] for i in range(N5)], outs[2:], thr)
                O.simd_code(G5[N5:], [sh[i] for i in range(N5)], tmp, thr)
                ok = all(np.array_equal(tmp[r_], sh[N5 + r_]) for r_ in range(t5.M))
                for a in range(t5.AZCount):
                    ia, _, _ = t5.LocalStripeInAZ(a)
                    O.simd_code(Lm5[l5:], [sh[i] for i in ia[:l5]], ltmp, thr)
                    ok = ok and np.array_equal(ltmp[0], sh[ia[l5]])
                return ok
            return f

        sh = [np.ascontiguousarray(h[i]) for i in range(tot5)]
        assert cpu_rep5(sh, thr)()
        rate_c5 = cpu_rate(cpu_rep5(sh, thr), cpu_secs)
        sat5 = cpu_saturated_rate(lambda w: cpu_rep5([x.copy() for x in sh], 1), cpu_secs, callers)
        c5["cpu_baseline"] = {"value": round(N5 * S5 * rate_c5 / 1e9, 3), "unit": "GB/s", "cores": thr, "kind": "port",
                              "sample": "one bid: reconstruct 2 data + 2 parity rows, global and 2 local verifies, repeated",
                              "saturated": {"value": round(N5 * S5 * sat5 / 1e9, 3), "unit": "GB/s", "cores": callers,
                                            "sample": f"{callers} single-threaded callers, one bid each"}}
    out["C5_EC16P20L2_repair_tasklet"] = c5
    del bm5, b5, gold5, cw5
    return out


if __name__ == "__main__":
    main()
