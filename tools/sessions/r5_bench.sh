# round-5 bench session: the driver's bench line (PMC traffic + CPU baseline), a kernel-trace profile
# of the same bench with the timed-region statistics, the shape sweep, and the N = 2 rehearsal
set -o pipefail
mkdir -p gpurun_out/r5c
export TMPDIR=/tmp
timeout -k 10 420 python bench.py > gpurun_out/r5c/bench.json 2> gpurun_out/r5c/bench.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 3 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5c/prof -o run -- python3 bench.py --no-cpu --no-pmc > gpurun_out/r5c/bench_prof.json 2> gpurun_out/r5c/bench_prof.err; rc=$?
echo "prof rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 3 ] || exit $rc
python tools/timed_region_stats.py gpurun_out/r5c/prof gpurun_out/r5c/bench_prof.json gpurun_out/r5c/timed_region_stats.txt
timeout -k 10 200 ./tools/gf_shapes > gpurun_out/r5c/shape_sweep.txt 2>&1 || exit $?
CFSEC_BENCH_SHARE_DEVICE=1 CFSEC_BENCH_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --no-cpu --no-pmc --op-seconds 0.5 > gpurun_out/r5c/bench_n2.json 2> gpurun_out/r5c/bench_n2.err; rc=$?
echo "n2 rc=$rc"
cat gpurun_out/r5c/timed_region_stats.txt | head -5
exit 0
