# Round 6, session O: the per-row form with W waves per stripe on every W-th tile (one checksum fold
# per wave and stripe): parity tests (the child runs EC12P4's route too), C4's put batch in each form,
# the shape sweep with EC12P4's route on.
set -o pipefail
mkdir -p gpurun_out/r6o
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bs_crc_fused.py \
  > gpurun_out/r6o/pytest_bs_crc.log 2>&1 || { tail -40 gpurun_out/r6o/pytest_bs_crc.log; exit 1; }
tail -1 gpurun_out/r6o/pytest_bs_crc.log
for v in 5 1 0; do
  echo "== CFSEC_BS_CRC=$v" >> gpurun_out/r6o/c4.txt
  CFSEC_BS_CRC=$v timeout -k 10 120 python tools/c4_crc_probe.py >> gpurun_out/r6o/c4.txt 2>&1 || exit $?
done
grep -E "==|us per call|all" gpurun_out/r6o/c4.txt
for v in 7 0; do
  echo "== CFSEC_BS_CRC=$v" >> gpurun_out/r6o/shapes.txt
  CFSEC_BS_CRC=$v timeout -k 10 200 ./tools/gf_shapes >> gpurun_out/r6o/shapes.txt 2>&1 || exit $?
done
grep -E "==|EC12P4|EC6P10L2 fused" gpurun_out/r6o/shapes.txt
exit 0
