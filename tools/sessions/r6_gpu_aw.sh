# Round 6, session AW: tests/test_gpu_bs_crc_tail.py with the pointer-table case.
set -o pipefail
mkdir -p gpurun_out/r6aw
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bs_crc_tail.py \
  > gpurun_out/r6aw/pytest.log 2>&1 || { tail -60 gpurun_out/r6aw/pytest.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/r6aw/pytest.log | tail -8
exit 0
