#!/usr/bin/env python3
"""bench.py -- EC12P4 encode + 4-erasure reconstruct throughput on MI355X.

Workload (BASELINE.json configs[1]/[2], one GPU): a batch of `--stripes` EC12P4
stripes of 64 MiB blobs (shard size S = ceil(64 MiB / 12) = 5,592,406 B), resident
in HBM with a 256-B shard pitch.  One step = one pass of the hot path over the batch:
  1. Encode       (cfsec_rs_encode_batch):      read 12*S, write 4*S per stripe
  2. Reconstruct  erased {0,1,2,3}, the worst-case dense decode
                  (cfsec_rs_reconstruct_batch): read 12*S, write 4*S per stripe
value = data bytes through the engine per second = 2 * 12 * S * stripes * n_gpus / step
time (each operation counts its stripe's 12*S data bytes once).  Multi-GPU: each rank
codes its own stripes (weak scaling, no collective on the data path).

    python bench.py [--gpus N --steps K --warmup W]
"""
from __future__ import annotations

import argparse
import ctypes
import csv
import glob
import json
import os
import shutil
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
HBM_PEAK_GBPS = 8000.0  # MI355X spec (MI355X_MICROARCH.md)
KERNEL = "gf_dy_kernel<12, 4, 4, (cfsec::MatVecMode)0, 0>"  # both step kernels: 12 -> 4 rows, 4x4-dyadic matrices


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--stripes", type=int, default=8, help="stripes per GPU per step")
    p.add_argument("--shard-size", type=int, default=S_DEFAULT)
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample length")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-pmc", action="store_true")
    p.add_argument("--graph", action="store_true", help="replay each step as a captured HIP graph")
    p.add_argument("--settle-ms", type=float, default=400.0, help="untimed load before warmup (clock ramp)")
    p.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    return p.parse_args()


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
def cpu_baseline(S, seconds):
    """klauspost-strategy restatement (oracle/cpu_simd.c) on the host: the same EC12P4 encode +
    4-erasure reconstruct of one stripe, repeated for ~`seconds`, with the reference's per-call
    worker cap (4 with GFNI, else 8; KRS/reedsolomon.go:551-557)."""
    import numpy as np

    from oracle import oracle as O

    feats = O.simd_features()
    threads = 4 if feats["gfni"] else 8
    rng = np.random.default_rng(0xCF5EC000)
    data = [rng.integers(0, 256, S, dtype=np.uint8) for _ in range(K_DATA)]
    parity = [np.zeros(S, np.uint8) for _ in range(M_PARITY)]
    full = O.build_matrix(K_DATA, K_DATA + M_PARITY)
    prow = full[K_DATA:]
    err, dec = O.invert(full[4:16])  # survivors 4..15 after erasing {0,1,2,3}
    assert err == 0
    drows = dec[:4]
    survivors = data[4:] + parity
    rebuilt = [np.zeros(S, np.uint8) for _ in range(4)]
    O.simd_code(prow, data, parity, threads)  # warm
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
    saturated = cpu_saturated(S, prow, drows, max(2.0, seconds / 2))
    return {
        "value": round(value, 3), "unit": "GB/s", "cores": threads, "kind": "port",
        "sample": (f"EC12P4 encode + erase{{0,1,2,3}} reconstruct of one S={S} stripe x{ops} "
                   f"({dt:.1f}s), klauspost v1.11.7 strategy restated in C "
                   f"({'AVX2 10x4+2x4 tiles' if kind == 1 else 'GFNI tiles'}), {threads} worker threads"),
        "host_cpus": os.cpu_count(),
        "features": feats,
        "saturated": saturated,
    }


def cpu_saturated(S, prow, drows, seconds):
    """BASELINE.md's second CPU mode: `callers` concurrent single-threaded callers, each coding its
    own EC12P4 stripe (encode + the {0,1,2,3} reconstruct), for ~`seconds`.  callers = the host's
    CPUs, capped at 16 (the GPU box's CPU share)."""
    import threading

    import numpy as np

    from oracle import oracle as O

    callers = max(1, min(16, os.cpu_count() or 1))
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
def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    S, nst = args.shard_size, args.stripes

    traffic, pmc_note = None, "skipped"
    if rank == 0 and world == 1 and not args.no_pmc and not args.pmc_child:
        traffic, pmc_note = pmc_traffic(args)  # before this process touches the GPU

    import torch

    from chubaofs_amd import reedsolomon

    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    total = K_DATA + M_PARITY
    pitch = (S + 255) // 256 * 256
    batch = torch.zeros((nst, total, pitch), dtype=torch.uint8, device=dev)
    for s in range(nst):  # seeded synthetic data, one generator per stripe
        g = torch.Generator(device=dev)
        g.manual_seed(0xCF5EC000 + rank * nst + s)
        batch[s, :K_DATA, :S] = torch.randint(0, 256, (K_DATA, S), generator=g, device=dev, dtype=torch.uint8)
    base = batch.data_ptr()
    ptrs = [base + (s * total + i) * pitch for s in range(nst) for i in range(total)]
    ptrs = (ctypes.c_void_p * len(ptrs))(*ptrs)  # marshalled once, reused by every launch
    enc = reedsolomon.New(K_DATA, M_PARITY, device=local_rank)
    stream = torch.cuda.Stream(device=dev)

    def step():
        enc.encode_batch(ptrs, S, nst, stream=stream)
        enc.reconstruct_batch(ptrs, S, nst, ERASED, stream=stream)

    if args.pmc_child:
        for _ in range(args.warmup + args.steps):
            step()
        torch.cuda.synchronize()
        return

    step()  # plans the reconstruct (inversion cache) before any timing or capture
    torch.cuda.synchronize()
    graph = None
    if args.graph:
        # optional: one step (two launches) captured into a HIP graph and replayed
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=stream):
            step()
        torch.cuda.synchronize()

    def run_step():
        if graph is None:
            step()
        else:
            with torch.cuda.stream(stream):
                graph.replay()

    def timed(fn, n):
        """Mean ms per call of fn over n back-to-back calls, one event pair on the launch
        stream: a timestamp between launches opens idle gaps in the queue (measured
        6-20 us on MI355X) that slow the next kernel, so per-launch events would time the
        harness, not the kernel."""
        t_s = time.perf_counter()
        while time.perf_counter() - t_s < 0.1:  # settle after the host-side checks' idle gap
            for _ in range(10):
                fn()
            torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(n):
            fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n

    # Settle: after idle the first ~100-200 launches run up to 10 % slower while the clocks
    # ramp (measured with tools/bench_env.py), so the device is loaded with the step for
    # --settle-ms before the W warmup steps.  Nothing from this phase is timed or counted.
    t_settle = time.perf_counter()
    while time.perf_counter() - t_settle < args.settle_ms / 1e3:
        for _ in range(10):
            run_step()
        torch.cuda.synchronize()
    for _ in range(args.warmup):
        run_step()
    torch.cuda.synchronize()
    golden = batch[:, :, :S].clone()

    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        run_step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    # both step kernels are gf_dy_kernel<12, 4, 4, kStore> moving the same algorithmic bytes
    avg_ms = ev0.elapsed_time(ev1) / (2 * args.steps)

    # correctness gate: the stripes are unchanged codewords after K reconstructs
    assert torch.equal(batch[:, :, :S], golden), "batch changed across reconstruct passes"
    # per-operation rates (outside the timed region)
    n_op = max(args.steps, 10)
    enc_ms = timed(lambda: enc.encode_batch(ptrs, S, nst, stream=stream), n_op)
    rec_ms = timed(lambda: enc.reconstruct_batch(ptrs, S, nst, ERASED, stream=stream), n_op)
    flags = torch.zeros(nst, dtype=torch.int32, device=dev)
    verify_ms = timed(lambda: enc.verify_batch(ptrs, S, nst, flags.data_ptr(), stream=stream), n_op)
    assert int(flags.sum().item()) == 0, "Verify failed after the timed region"
    # Encode + crc32.ChecksumIEEE of all 16 shards (access/stream_put.go:249-253), fused into the
    # coding kernel: same algorithmic bytes as the encode
    crcs = torch.zeros(nst * total, dtype=torch.int32, device=dev)
    crc_ms = timed(lambda: enc.encode_crc_batch(ptrs, S, nst, crcs.data_ptr(), stream=stream), n_op)
    # Blobnode's write path frames each shard in 64 KiB crc32block blocks and takes the shard's
    # checksum on the way (core/storage/datafile.go:345-373); its read path checks and unframes them
    # (datafile.go:406-426).  All 16 shards of every stripe in one framing / one checking launch.
    from chubaofs_amd import crc32block
    nsh = nst * total
    flen = crc32block.EncodeSize(S)
    # one 256-byte-aligned row per framed shard / unframed shard, like the stripes' rows
    framed = torch.empty((nsh, (flen + 255) // 256 * 256), dtype=torch.uint8, device=dev)
    unframed = torch.empty((nsh, pitch), dtype=torch.uint8, device=dev)
    fptrs = (ctypes.c_void_p * nsh)(*[framed[i].data_ptr() for i in range(nsh)])
    uptrs = (ctypes.c_void_p * nsh)(*[unframed[i].data_ptr() for i in range(nsh)])
    fcrc = torch.zeros(nsh, dtype=torch.int32, device=dev)
    fbad = torch.zeros(nsh, dtype=torch.int32, device=dev)
    blk_enc_ms = timed(lambda: crc32block.encode_batch(ptrs, fptrs, S, shard_crcs_ptr=fcrc.data_ptr(),
                                                       stream=stream), n_op)
    blk_dec_ms = timed(lambda: crc32block.decode_batch(fptrs, uptrs, S, fbad.data_ptr(), stream=stream), n_op)
    assert bool((fbad == -1).all().item()), "crc32block check failed on freshly framed shards"
    assert torch.equal(unframed[:, :S].reshape(nst, total, S), batch[:, :, :S]), "crc32block round trip differs"
    blk_bytes = nsh * (S + flen)  # read the payload and write the frames, or the reverse
    del framed, unframed

    data_bytes = K_DATA * S * nst
    launch_bytes = (K_DATA + M_PARITY) * S * nst  # algorithmic bytes per launch (read 12S + write 4S)
    achieved = launch_bytes / (avg_ms * 1e-3) / 1e9
    value = 2 * data_bytes * world * args.steps / elapsed / 1e9

    if rank != 0:
        if world > 1:
            torch.distributed.destroy_process_group()
        return
    cpu = None
    if world == 1 and not args.no_cpu:
        cpu = cpu_baseline(S, args.cpu_seconds)
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
            "code_mode": "EC12P4", "shard_size": S, "shard_pitch": pitch, "stripes_per_gpu": nst,
            "erased": ERASED, "parallelism": f"stripes sharded over {world} GPU(s), no collective",
            "value_def": "2 * 12 * S * stripes * n_gpus / step time (encode and reconstruct each count the stripe's data once)",
        },
        "roofline": {
            "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 4),
            "traffic": None if traffic is None else int(traffic),
            "kernel": "gf_dy_kernel<12, 4, 4, kStore, 0> (encode and reconstruct launches: both matrices are 4x4-dyadic)",
            "algorithmic_bytes_per_launch": launch_bytes,
            "avg_launch_ms": round(avg_ms, 4),
            "launch_timing": ("HIP event pair on the launch stream around the timed region / launches"
                              + (" (graph replay)" if graph is not None else "")),
            "traffic_note": pmc_note if traffic is None else "rocprofv3 (2*FETCH_SIZE + WRITE_SIZE)*1024, per launch",
            "cache_note": ("the step alternates encode and reconstruct over the same stripes: each reads the "
                           "4 rows the other just wrote (4*S*stripes = 179 MB, under the 256 MB Infinity Cache), "
                           "and with sc1 output stores part of that is served from the cache; the same kernels "
                           "repeated back to back on one operation (no reuse) give encode_roofline_frac / "
                           "reconstruct_roofline_frac"),
        },
        "encode_data_GBps": round(data_bytes / (enc_ms * 1e-3) / 1e9, 1),
        "encode_roofline_frac": round(launch_bytes / (enc_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
        "reconstruct_data_GBps": round(data_bytes / (rec_ms * 1e-3) / 1e9, 1),
        "reconstruct_roofline_frac": round(launch_bytes / (rec_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
        "verify_data_GBps": round(data_bytes / (verify_ms * 1e-3) / 1e9, 1),
        "verify_roofline_frac": round(launch_bytes / (verify_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
        "encode_crc_data_GBps": round(data_bytes / (crc_ms * 1e-3) / 1e9, 1),
        "encode_crc_roofline_frac": round(launch_bytes / (crc_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
        "crc32block_encode_data_GBps": round(nsh * S / (blk_enc_ms * 1e-3) / 1e9, 1),
        "crc32block_encode_roofline_frac": round(blk_bytes / (blk_enc_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
        "crc32block_decode_data_GBps": round(nsh * S / (blk_dec_ms * 1e-3) / 1e9, 1),
        "crc32block_decode_roofline_frac": round(blk_bytes / (blk_dec_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4),
        "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
