"""HBM bytes per launch of every kernel in two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; KiB;
FETCH_SIZE doubled for gfx950's 16-B/lane streams as bench.py does), beside the launch's algorithmic
bytes when given:  python tools/pmc_kernel_traffic.py <fetch dir> <write dir> [name=bytes ...]"""
import csv
import glob
import os
import sys
from collections import defaultdict


def per_kernel(d, ctr):
    acc = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name", ctr) == ctr:
                    acc[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()}


fetch, n = per_kernel(sys.argv[1], "FETCH_SIZE")
write, _ = per_kernel(sys.argv[2], "WRITE_SIZE")
alg = dict(a.split("=", 1) for a in sys.argv[3:])
for k in sorted(fetch, key=lambda k: -fetch[k]):
    if k not in write:
        continue
    t = (2.0 * fetch[k] + write[k]) * 1024.0
    short = k.replace("(anonymous namespace)::", "").split("(")[0][-70:]
    want = next((float(v) for s, v in alg.items() if s in k), None)
    extra = f"  algorithmic {want:.0f} B: x{t / want:.3f}" if want else ""
    print(f"{short:70s} n={n[k]:4d}  read {2 * fetch[k] * 1024:.0f} B  write {write[k] * 1024:.0f} B  total {t:.0f} B{extra}")
