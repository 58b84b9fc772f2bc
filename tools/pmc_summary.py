#!/usr/bin/env python3
"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel name (mean per dispatch)."""
import csv
import glob
import sys
from collections import defaultdict

rows = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = defaultdict(lambda: defaultdict(list))
for r in rows:
    agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, ctrs in agg.items():
    short = k.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")[-70:]
    print(short)
    for c, v in sorted(ctrs.items()):
        print(f"    {c:28s} n={len(v):5d} mean={sum(v) / len(v):.4g}")
