# Round 6, session AO: the full GPU suite with EC6P6 and EC16P4 on the bit-sliced route (default 119).
set -o pipefail
mkdir -p gpurun_out/r6ao
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r6ao/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r6ao/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r6ao/pytest_gpu.log
exit 0
