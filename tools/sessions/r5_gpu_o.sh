# round-5 session O: device timeline of the scattered C5 calls (kernels + copies)
set -o pipefail
mkdir -p gpurun_out/r5
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
C5_REPS=30 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r5/scat_trace -o scat -- python3 tools/c5_scatter_probe.py > gpurun_out/r5/scat_trace.log 2>&1 || exit $?
n=$(python3 tools/trace_timeline.py gpurun_out/r5/scat_trace --count 100000 | wc -l)
python3 tools/trace_timeline.py gpurun_out/r5/scat_trace --skip $((n - 40)) --count 40 > gpurun_out/r5/scat_timeline.txt
python3 tools/trace_timeline.py gpurun_out/r5/scat_trace --skip $((n / 2)) --count 40 >> gpurun_out/r5/scat_timeline.txt
cat gpurun_out/r5/scat_timeline.txt; tail -5 gpurun_out/r5/scat_trace.log
