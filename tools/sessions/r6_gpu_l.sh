# Round 6, session L: the plane-residue form of C4's fused encode + 18 checksums (gf_bs_crc.hip
# bc_w_kernel): its parity tests (and, in a child, the per-row form and EC12P4's route), the checksum
# suites, then C4's put batch in every form and the shape sweep.
set -o pipefail
mkdir -p gpurun_out/r6l
export TMPDIR=/tmp
CFSEC_BS_CRC=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bs_crc_fused.py \
  > gpurun_out/r6l/pytest_bs_crc_w.log 2>&1 || { tail -40 gpurun_out/r6l/pytest_bs_crc_w.log; exit 1; }
tail -1 gpurun_out/r6l/pytest_bs_crc_w.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bs_crc_fused.py \
  > gpurun_out/r6l/pytest_bs_crc.log 2>&1 || { tail -40 gpurun_out/r6l/pytest_bs_crc.log; exit 1; }
tail -1 gpurun_out/r6l/pytest_bs_crc.log
CFSEC_BS_CRC=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_crc.py \
  tests/test_gpu_batch.py -k "crc" > gpurun_out/r6l/pytest_crc.log 2>&1 || { tail -40 gpurun_out/r6l/pytest_crc.log; exit 1; }
tail -1 gpurun_out/r6l/pytest_crc.log
for v in 1 5 0 w3; do
  lib=chubaofs_amd/libcfsec.so; m=$v; [ $v = w3 ] && { lib=probes_bin/bw_wpe3/libcfsec.so; m=1; }
  echo "== CFSEC_BS_CRC=$v" >> gpurun_out/r6l/c4.txt
  CFSEC_LIB_PATH=$PWD/$lib CFSEC_BS_CRC=$m timeout -k 10 120 python tools/c4_crc_probe.py >> gpurun_out/r6l/c4.txt 2>&1 || exit $?
done
grep -E "==|us per call|all" gpurun_out/r6l/c4.txt
CFSEC_BS_CRC=1 timeout -k 10 200 ./tools/gf_shapes > gpurun_out/r6l/shapes.txt 2>&1 || exit $?
grep -E "EC12P4|EC6P10L2 fused" gpurun_out/r6l/shapes.txt
exit 0
