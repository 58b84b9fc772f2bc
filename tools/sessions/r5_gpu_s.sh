# round-5 session S: which kernels the probe's shipped (8, 1) launch runs, and their durations
set -o pipefail
mkdir -p gpurun_out/r5
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/c4lprof -o c4l -- tools/c4l_pattern_probe > gpurun_out/r5/c4lprof.log 2>&1 || exit $?
cut -d, -f1-4 gpurun_out/r5/c4lprof/c4l_kernel_stats.csv | cut -c1-200
