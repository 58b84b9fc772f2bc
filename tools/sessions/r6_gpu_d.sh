# Round 6, session D: C4's fused LRC encode + 18 checksums -- lookup kernel with 16-byte entries
# (default), its 5-bit output-checksum form (r6_out5, also EC12P4's), deeper lookup pipelining
# (r6_pipew), and the round-5 v_perm form (CFSEC_CRC_LDS12=0); every probe run checks all 48 blobs'
# parity and words; then the shape sweep of each library.
set -o pipefail
mkdir -p gpurun_out/r6d
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_batch.py \
  tests/test_gpu_crc.py -k "crc" > gpurun_out/r6d/pytest_crc.log 2>&1 || { tail -40 gpurun_out/r6d/pytest_crc.log; exit 1; }
tail -1 gpurun_out/r6d/pytest_crc.log
CFSEC_LIB_PATH=$PWD/probes_bin/r6_out5/libcfsec.so timeout -k 10 300 python -u -m pytest -q --timeout 120 \
  --timeout-method thread -m gpu tests/test_gpu_batch.py tests/test_gpu_crc.py -k "crc" > gpurun_out/r6d/pytest_out5.log 2>&1 \
  || { tail -40 gpurun_out/r6d/pytest_out5.log; exit 1; }
tail -1 gpurun_out/r6d/pytest_out5.log
for i in 1 2; do
  timeout -k 10 120 python3 tools/c4_crc_probe.py > gpurun_out/r6d/c4_lds12_$i.txt 2>&1 && \
  CFSEC_LIB_PATH=$PWD/probes_bin/r6_out5/libcfsec.so timeout -k 10 120 python3 tools/c4_crc_probe.py > gpurun_out/r6d/c4_out5_$i.txt 2>&1 && \
  CFSEC_LIB_PATH=$PWD/probes_bin/r6_pipew/libcfsec.so timeout -k 10 120 python3 tools/c4_crc_probe.py > gpurun_out/r6d/c4_pipew_$i.txt 2>&1 && \
  CFSEC_CRC_LDS12=0 timeout -k 10 120 python3 tools/c4_crc_probe.py > gpurun_out/r6d/c4_vperm_$i.txt 2>&1 || exit $?
done
for f in gpurun_out/r6d/c4_*.txt; do echo "== $f"; grep "us per call\|blobs" $f | tr '\n' ' '; echo; done
timeout -k 10 200 ./tools/gf_shapes > gpurun_out/r6d/shapes_cur.txt 2>&1 && \
timeout -k 10 200 ./probes_bin/r6_out5/gf_shapes > gpurun_out/r6d/shapes_out5.txt 2>&1 && \
timeout -k 10 200 ./probes_bin/r6_pipew/gf_shapes > gpurun_out/r6d/shapes_pipew.txt 2>&1 || exit $?
grep "EC12P4\|EC16P4\|EC6P10L2\|EC6P6" gpurun_out/r6d/shapes_*.txt
