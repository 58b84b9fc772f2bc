# Round 6, session J: the full GPU suite + smoke (pageable small calls now staged through page-locked
# memory), the C-ABI latency tool, then the bench session recipe: the driver's bench line, a
# kernel-trace profile of the same bench with the timed-region statistics, the shape sweep.
set -o pipefail
mkdir -p gpurun_out/r6j
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r6j/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r6j/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r6j/pytest_gpu.log
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' 2>&1 | tail -1
timeout -k 10 120 ./tools/seg_latency 200 null > gpurun_out/r6j/seg_latency_null.json 2>&1 || exit $?
cat gpurun_out/r6j/seg_latency_null.json
timeout -k 10 500 python bench.py > gpurun_out/r6j/bench.json 2> gpurun_out/r6j/bench.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 3 ] || { tail -20 gpurun_out/r6j/bench.err; exit $rc; }
timeout -k 10 450 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6j/prof -o run -- python3 bench.py --no-cpu --no-pmc > gpurun_out/r6j/bench_prof.json 2> gpurun_out/r6j/bench_prof.err; rc=$?
echo "prof rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 3 ] || exit $rc
python tools/timed_region_stats.py gpurun_out/r6j/prof gpurun_out/r6j/bench_prof.json gpurun_out/r6j/timed_region_stats.txt
head -5 gpurun_out/r6j/timed_region_stats.txt
timeout -k 10 200 ./tools/gf_shapes > gpurun_out/r6j/shape_sweep.txt 2>&1 || exit $?
exit 0
