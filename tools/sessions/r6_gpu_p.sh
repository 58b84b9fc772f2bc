# Round 6, session P: the per-row form's lane fold by recursive halving (lookups instead of a 32-column
# basis per register): parity tests, C4's put batch, and the same structure without the checksum
# lookups (probe, wrong words), the shape sweep with EC12P4's route on.
set -o pipefail
mkdir -p gpurun_out/r6p
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bs_crc_fused.py \
  > gpurun_out/r6p/pytest_bs_crc.log 2>&1 || { tail -40 gpurun_out/r6p/pytest_bs_crc.log; exit 1; }
tail -1 gpurun_out/r6p/pytest_bs_crc.log
for v in 5 p3; do
  lib=chubaofs_amd/libcfsec.so; [ $v = p3 ] && lib=probes_bin/pr_probe3/libcfsec.so
  echo "== $v" >> gpurun_out/r6p/c4.txt
  CFSEC_LIB_PATH=$PWD/$lib CFSEC_BS_CRC=5 timeout -k 10 120 python tools/c4_crc_probe.py >> gpurun_out/r6p/c4.txt 2>&1
  rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
grep -E "==|us per call|all" gpurun_out/r6p/c4.txt
CFSEC_BS_CRC=7 timeout -k 10 200 ./tools/gf_shapes > gpurun_out/r6p/shapes.txt 2>&1 || exit $?
grep -E "EC12P4|EC6P10L2 fused" gpurun_out/r6p/shapes.txt
exit 0
