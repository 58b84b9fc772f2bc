# round-5 session A: stale-DMA probe (tools/r5_probe1.sh), then the new concurrency tests
set -o pipefail
mkdir -p gpurun_out/r5
bash tools/r5_probe1.sh > gpurun_out/r5/probe1.log 2>&1; prc=$?
cat gpurun_out/r5/probe1.log
[ $prc -eq 0 ] || exit $prc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_concurrency.py > gpurun_out/r5/test_concurrency.log 2>&1; rc=$?
tail -15 gpurun_out/r5/test_concurrency.log
exit $rc
