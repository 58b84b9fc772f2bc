# One GPU session: GPU tests, smoke, the driver's bench line, a kernel-trace profile of the same
# bench with the timed-region statistics.  Every GPU step has its own time limit; the first
# failure ends the script (set -e).
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
python - > gpurun_out/host.txt <<'PY'
import os
print("os.cpu_count", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))
for f in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/memory.max"):
    try:
        print(f, open(f).read().strip())
    except OSError as e:
        print(f, e)
PY
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu --no-pmc > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
python tools/timed_region_stats.py gpurun_out/prof gpurun_out/bench_prof.json gpurun_out/timed_region_stats.txt
cat gpurun_out/smoke.log gpurun_out/bench.json
