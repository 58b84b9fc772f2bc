# Round 6, session T: the input rows' Horner registers in LDS for k > 8 (EC16P20(L2): 79 -> 33 spilled
# VGPRs; EC12P4 at 3 waves per SIMD): parity tests (child: every route), the shape sweep per route mask.
set -o pipefail
mkdir -p gpurun_out/r6t
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_bs_crc_fused.py \
  > gpurun_out/r6t/pytest_bs_crc.log 2>&1 || { tail -40 gpurun_out/r6t/pytest_bs_crc.log; exit 1; }
tail -1 gpurun_out/r6t/pytest_bs_crc.log
for v in 7 0; do
  echo "== CFSEC_BS_CRC=$v" >> gpurun_out/r6t/shapes.txt
  CFSEC_BS_CRC=$v timeout -k 10 200 ./tools/gf_shapes >> gpurun_out/r6t/shapes.txt 2>&1 || exit $?
done
grep -E "==|EC16P20 global|EC16P20L2 fused|EC12P4 encode|EC6P10L2 fused" gpurun_out/r6t/shapes.txt
exit 0
