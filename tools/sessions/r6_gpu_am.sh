# Round 6, session AM: GPU tests of the bit-sliced kernel's tail waves (tests/test_gpu_bs_crc_tail.py)
# and the fused-route module.
set -o pipefail
mkdir -p gpurun_out/r6am
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bs_crc_tail.py \
  tests/test_gpu_bs_crc_fused.py > gpurun_out/r6am/pytest.log 2>&1 || { tail -60 gpurun_out/r6am/pytest.log; exit 1; }
grep -E "tail|passed|failed" gpurun_out/r6am/pytest.log | tail -12
exit 0
