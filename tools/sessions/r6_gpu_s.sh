# Round 6, session S: the bit-sliced fused encode + checksums for the 16 + 20 code (EC16P20 / EC16P20L2,
# CFSEC_BS_CRC bit 2; 256 VGPRs with 79 spilled at 2 waves per SIMD): parity tests in the child
# (CFSEC_BS_CRC=7), the shape sweep with and without the route.
set -o pipefail
mkdir -p gpurun_out/r6s
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_bs_crc_fused.py \
  > gpurun_out/r6s/pytest_bs_crc.log 2>&1 || { tail -40 gpurun_out/r6s/pytest_bs_crc.log; exit 1; }
tail -1 gpurun_out/r6s/pytest_bs_crc.log
for v in 5 1; do
  echo "== CFSEC_BS_CRC=$v" >> gpurun_out/r6s/shapes.txt
  CFSEC_BS_CRC=$v timeout -k 10 200 ./tools/gf_shapes >> gpurun_out/r6s/shapes.txt 2>&1 || exit $?
done
grep -E "==|EC16P20|EC12P4 encode 64|EC6P10L2 fused" gpurun_out/r6s/shapes.txt
exit 0
