# Round 6, session AD: the bit-sliced fused kernel's remainder tiles (tps mod W) as one tile per
# extra wave (CFSEC_BC_TAIL, percent of W; 0: the W-strided rounds as before) -- parity tests, then
# C4's put batch at 320 / 321 / 342 tiles per row, and two other modes, with and without.
set -o pipefail
mkdir -p gpurun_out/r6ad
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_bs_crc_fused.py \
  > gpurun_out/r6ad/pytest_bs_crc.log 2>&1 || { tail -40 gpurun_out/r6ad/pytest_bs_crc.log; exit 1; }
tail -1 gpurun_out/r6ad/pytest_bs_crc.log
for S in 699051 657000; do
  for v in 0 100 50; do
    echo "== EC6P10L2 S=$S CFSEC_BC_TAIL=$v" >> gpurun_out/r6ad/tail.txt
    CFSEC_BC_TAIL=$v timeout -k 10 120 python tools/lrc_crc_probe.py EC6P10L2 $S 48 >> gpurun_out/r6ad/tail.txt 2>&1 || exit $?
  done
done
for m in EC6P6L9 EC12P9 EC16P20L2; do
  for v in 0 100; do
    echo "== $m CFSEC_BC_TAIL=$v" >> gpurun_out/r6ad/tail.txt
    CFSEC_BC_TAIL=$v timeout -k 10 120 python tools/lrc_crc_probe.py $m 699051 32 >> gpurun_out/r6ad/tail.txt 2>&1 || exit $?
  done
done
grep -E "==|us per call|all" gpurun_out/r6ad/tail.txt
exit 0
