"""Timeline of a rocprofv3 --kernel-trace --memory-copy-trace run (csv output): every kernel dispatch
and copy in start order, with durations and the gap to the previous operation's end, for the ops
whose start falls in the [--from, --to) fraction of the trace (dev tool):
  python3 tools/trace_timeline.py <dir> [--skip N] [--count N]"""
import csv
import glob
import os
import sys

d = sys.argv[1]
skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 0
count = int(sys.argv[sys.argv.index("--count") + 1]) if "--count" in sys.argv else 60
ops = []
for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:90]))
for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                    "COPY " + r.get("Direction", "") + " " + r.get("Size", r.get("Bytes", ""))))
ops.sort()
prev = None
for s, e, n in ops[skip:skip + count]:
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    print(f"{gap:9.2f} us gap  {(e - s) / 1e3:9.2f} us  {n}")
    prev = e
