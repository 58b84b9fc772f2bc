# Round 6, session K: the bit-sliced fused encode + checksum kernels (gf_bs_crc.hip) -- their parity
# tests and the neighbouring checksum suites, then C4's put batch and the shape sweep with and without
# them (CFSEC_BS_CRC=0: the lookup-product kernels).
set -o pipefail
mkdir -p gpurun_out/r6k
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bs_crc_fused.py \
  > gpurun_out/r6k/pytest_bs_crc.log 2>&1 || { tail -40 gpurun_out/r6k/pytest_bs_crc.log; exit 1; }
tail -1 gpurun_out/r6k/pytest_bs_crc.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_crc.py \
  tests/test_gpu_batch.py -k "crc" > gpurun_out/r6k/pytest_crc.log 2>&1 || { tail -40 gpurun_out/r6k/pytest_crc.log; exit 1; }
tail -1 gpurun_out/r6k/pytest_crc.log
for v in 3 0; do
  echo "== CFSEC_BS_CRC=$v" >> gpurun_out/r6k/c4_crc.txt
  CFSEC_BS_CRC=$v timeout -k 10 120 python tools/c4_crc_probe.py >> gpurun_out/r6k/c4_crc.txt 2>&1 || exit $?
  echo "== CFSEC_BS_CRC=$v" >> gpurun_out/r6k/shapes.txt
  CFSEC_BS_CRC=$v timeout -k 10 200 ./tools/gf_shapes >> gpurun_out/r6k/shapes.txt 2>&1 || exit $?
done
cat gpurun_out/r6k/c4_crc.txt
grep -E "==|EC12P4|EC6P10L2 fused" gpurun_out/r6k/shapes.txt
exit 0
