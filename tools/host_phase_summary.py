"""Median per phase of CFSEC_HOST_TIMING's stderr lines, grouped by the '--- <call>' markers that
tools/host_timing.py writes before each timed call (dev tool):
  python3 tools/host_phase_summary.py timing.txt"""
import collections
import re
import statistics
import sys

calls = collections.OrderedDict()
cur = None
for line in open(sys.argv[1]):
    if line.startswith("--- "):
        cur = line[4:].strip()
        calls.setdefault(cur, collections.OrderedDict())
        continue
    m = re.match(r"cfsec host (.*?)\s+([0-9.]+) us", line.rstrip())
    if m and cur:
        calls[cur].setdefault(m.group(1), []).append(float(m.group(2)))
for call, phases in calls.items():
    print(f"== {call}")
    for name, v in phases.items():
        print(f"   {name:34s} median {statistics.median(v):8.1f} us  (n={len(v)})")
