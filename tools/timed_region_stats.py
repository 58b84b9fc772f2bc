#!/usr/bin/env python3
"""Per-kernel statistics of bench.py's timed region from a rocprofv3 kernel trace.

bench.py reports roofline.timed_dispatches = [first, last): the indices, in dispatch order, of its
timed launches among the launches of the step kernel.  This script takes the rocprofv3
`--kernel-trace --output-format csv` output of the same command, orders that kernel's dispatches
by start time and summarises exactly those launches (no settle, warmup or post-timing launches).

    python tools/timed_region_stats.py <trace dir> <bench json line file> [out.txt]
"""
import csv
import glob
import json
import os
import statistics
import sys


def main():
    tdir, bench_out = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else None
    line = [l for l in open(bench_out) if l.startswith("{")][-1]
    b = json.loads(line)
    first, last = b["roofline"]["timed_dispatches"]
    want = b["roofline"].get("kernel_match", "gf_dy_kernel<12, 4, 4, (cfsec::MatVecMode)0, 0>").replace(" ", "")
    rows = []
    for f in glob.glob(os.path.join(tdir, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows += [r for r in csv.DictReader(fh) if want in r["Kernel_Name"].replace(" ", "")]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    sel = rows[first:last]
    if len(sel) != last - first:
        raise SystemExit(f"trace has {len(rows)} step-kernel dispatches, timed range [{first}, {last}) does not fit")
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in sel]  # us
    span = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e3
    bytes_ = b["roofline"]["algorithmic_bytes_per_launch"]
    mean = statistics.mean(dur)
    txt = [
        f"kernel: {sel[0]['Kernel_Name']}",
        f"timed dispatches [{first}, {last}) of {len(rows)} in the trace",
        f"launches: {len(dur)}  mean {mean:.2f} us  median {statistics.median(dur):.2f}  min {min(dur):.2f}  max {max(dur):.2f}",
        f"first start -> last end: {span:.1f} us over {b['steps']} steps = {span / b['steps']:.2f} us/step "
        f"(bench ms_per_step {b['ms_per_step'] * 1e3:.2f} us, bench avg_launch {b['roofline']['avg_launch_ms'] * 1e3:.2f} us)",
        f"algorithmic bytes per launch {bytes_}: {bytes_ / (mean * 1e-6) / 1e9:.1f} GB/s = "
        f"{bytes_ / (mean * 1e-6) / 1e9 / 8000:.4f} of 8 TB/s (mean launch duration)",
        f"check: 2 x mean launch = {2 * mean:.2f} us <= ms_per_step {b['ms_per_step'] * 1e3:.2f} us: "
        f"{2 * mean <= b['ms_per_step'] * 1e3}",
    ]
    text = "\n".join(txt) + "\n"
    print(text, end="")
    if out:
        with open(out, "w") as fh:
            fh.write(text)


if __name__ == "__main__":
    main()
