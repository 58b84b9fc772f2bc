# round-5 session I: scattered C5 calls with the waiting table ring, the bs tests, and the C4 / C5
# synchronous calls' host phases after the null-stream fast path
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_concurrency.py tests/test_gpu_batch.py -k "scattered or concurrency or two_streams or waits" > gpurun_out/r5/test_ring.log 2>&1; rc=$?
tail -2 gpurun_out/r5/test_ring.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/c5_scatter_probe.py > gpurun_out/r5/c5_scatter.txt 2>&1 && \
CFSEC_HOST_TIMING=1 timeout -k 10 300 python3 tools/host_timing.py > gpurun_out/r5/host_timing2.txt 2> gpurun_out/r5/host_timing2.err
rc=$?
cat gpurun_out/r5/c5_scatter.txt gpurun_out/r5/host_timing2.txt
grep -A12 -- '--- C4 local reconstruct_batch$' gpurun_out/r5/host_timing2.err | tail -13
exit $rc
