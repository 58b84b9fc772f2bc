# Round 6, session AI: the checksum pass kernel (crc32_horner_kernel) with its first tiles' loads
# issued before the step table is staged and 16 tiles in flight per thread -- its GPU tests, then
# C5's tasklet with / without checksums on the old kernel, the new order with 8 ahead, and the new
# kernel (the shipped build), alternated.
set -o pipefail
mkdir -p gpurun_out/r6ai
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_crc.py tests/test_gpu_batch.py \
  -k "crc" > gpurun_out/r6ai/pytest_crc.log 2>&1 || { tail -40 gpurun_out/r6ai/pytest_crc.log; exit 1; }
tail -1 gpurun_out/r6ai/pytest_crc.log
for lib in probes_bin/crc_old/libcfsec.so probes_bin/crc_a8/libcfsec.so chubaofs_amd/libcfsec.so probes_bin/crc_old/libcfsec.so probes_bin/crc_a8/libcfsec.so chubaofs_amd/libcfsec.so; do
  echo "== $lib" >> gpurun_out/r6ai/c5.txt
  CFSEC_LIB_PATH=$PWD/$lib timeout -k 10 120 python tools/c5_crc_probe.py >> gpurun_out/r6ai/c5.txt 2>&1 || { cat gpurun_out/r6ai/c5.txt; exit 1; }
done
grep -v amdgpu.ids gpurun_out/r6ai/c5.txt
exit 0
