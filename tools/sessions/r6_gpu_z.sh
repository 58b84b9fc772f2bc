# Round 6, session Z: the bit-sliced fused encode + checksums for the other RS modes (EC6P8, EC6P10,
# EC12P9, EC15P12, EC10P4; CFSEC_BS_CRC bit 4): parity tests (the child runs every route), the shape
# sweep with and without them.
set -o pipefail
mkdir -p gpurun_out/r6z
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_bs_crc_fused.py \
  > gpurun_out/r6z/pytest_bs_crc.log 2>&1 || { tail -40 gpurun_out/r6z/pytest_bs_crc.log; exit 1; }
tail -1 gpurun_out/r6z/pytest_bs_crc.log
for v in 21 0; do
  echo "== CFSEC_BS_CRC=$v" >> gpurun_out/r6z/shapes.txt
  CFSEC_BS_CRC=$v timeout -k 10 200 ./tools/gf_shapes >> gpurun_out/r6z/shapes.txt 2>&1 || exit $?
done
cat gpurun_out/r6z/shapes.txt
exit 0
