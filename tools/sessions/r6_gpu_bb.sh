# Round 6, session BB: the GPU suite with every bit-sliced checksum route off (CFSEC_BS_CRC=0: the
# lookup-product / v_perm fused kernels and the separate pass, the fallbacks the routes replaced),
# minus the two modules that assert the bit-sliced routes ran.
set -o pipefail
mkdir -p gpurun_out/r6bb
export TMPDIR=/tmp
CFSEC_BS_CRC=0 timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ \
  --ignore=tests/test_gpu_bs_crc_fused.py --ignore=tests/test_gpu_bs_crc_tail.py \
  > gpurun_out/r6bb/pytest_gpu_mask0.log 2>&1 || { tail -40 gpurun_out/r6bb/pytest_gpu_mask0.log; exit 1; }
tail -1 gpurun_out/r6bb/pytest_gpu_mask0.log
exit 0
