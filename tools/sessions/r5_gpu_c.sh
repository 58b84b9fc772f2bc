# round-5 session C: the repair-pass checksums (gf_bs16.hip CRC launches): tests, then C5 per-call
# times with / without checksums (fused, and CFSEC_BATCH_FUSED_CRC=0: the separate pass) and a
# kernel trace of the fused call
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bs_crc.py tests/test_gpu_concurrency.py > gpurun_out/r5/test_bs_crc.log 2>&1; rc=$?
tail -22 gpurun_out/r5/test_bs_crc.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/c5_crc_probe.py > gpurun_out/r5/c5_crc_fused.txt 2>&1 && \
CFSEC_BATCH_FUSED_CRC=0 timeout -k 10 120 python3 tools/c5_crc_probe.py > gpurun_out/r5/c5_crc_separate.txt 2>&1 && \
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/c5prof -o run --output-format csv -- python3 tools/c5_crc_probe.py > gpurun_out/r5/c5prof.log 2>&1
rc=$?
cat gpurun_out/r5/c5_crc_fused.txt gpurun_out/r5/c5_crc_separate.txt
find gpurun_out/r5/c5prof -name '*kernel_stats.csv' -exec cat {} \; | cut -c1-220 | head -12
exit $rc
