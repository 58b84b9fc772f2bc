# round-5 session D: the repair-pass checksums by read-back (tests + C5 per-call times), and the
# blocked tile mapping alone on the plain repair kernel (probes_bin/r5_blocked)
set -o pipefail
mkdir -p gpurun_out/r5
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bs_crc.py > gpurun_out/r5/test_bs_crc2.log 2>&1; rc=$?
tail -3 gpurun_out/r5/test_bs_crc2.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 120 python3 tools/c5_crc_probe.py > gpurun_out/r5/c5_crc_readback_$i.txt 2>&1 && \
CFSEC_BATCH_FUSED_CRC=0 timeout -k 10 120 python3 tools/c5_crc_probe.py > gpurun_out/r5/c5_crc_separate_$i.txt 2>&1 && \
CFSEC_LIB_PATH=probes_bin/r5_blocked/libcfsec.so CFSEC_BATCH_FUSED_CRC=0 timeout -k 10 120 python3 tools/c5_crc_probe.py > gpurun_out/r5/c5_blocked_$i.txt 2>&1 || exit $?
done
for f in gpurun_out/r5/c5_crc_readback_*.txt gpurun_out/r5/c5_crc_separate_*.txt gpurun_out/r5/c5_blocked_*.txt; do echo "== $f"; grep 'per call' $f; done
