# Round 6, session AA: the bit-sliced fused encode + checksums for the other LRC modes (EC6P3L3,
# EC4P4L2, EC6P6L9, EC6P8L10) and the wide ones' plain encodes (bit 5): parity tests, their put
# batches with and without the routes.
set -o pipefail
mkdir -p gpurun_out/r6aa
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_bs_crc_fused.py \
  tests/test_gpu_lrc_oracle.py > gpurun_out/r6aa/pytest_bs_crc.log 2>&1 || { tail -40 gpurun_out/r6aa/pytest_bs_crc.log; exit 1; }
tail -1 gpurun_out/r6aa/pytest_bs_crc.log
for m in EC6P3L3 EC4P4L2 EC6P6L9 EC6P8L10; do
  for v in 53 21; do
    echo "== $m CFSEC_BS_CRC=$v" >> gpurun_out/r6aa/lrc.txt
    CFSEC_BS_CRC=$v timeout -k 10 120 python tools/lrc_crc_probe.py $m 699051 32 >> gpurun_out/r6aa/lrc.txt 2>&1 || exit $?
  done
done
grep -E "==|us per call|all" gpurun_out/r6aa/lrc.txt
exit 0
