# Round 6, session C: C4's fused LRC encode + 18 checksums on the lookup-product kernel with 16-byte
# entries -- GPU tests of the checksum paths, then the C4 probe A/B (CFSEC_CRC_LDS12=0: the v_perm form)
set -o pipefail
mkdir -p gpurun_out/r6c
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_batch.py \
  tests/test_gpu_crc.py tests/test_gpu_lrc_oracle.py -k "crc or lrc or LRC" > gpurun_out/r6c/pytest_crc.log 2>&1 \
  || { tail -40 gpurun_out/r6c/pytest_crc.log; exit 1; }
tail -1 gpurun_out/r6c/pytest_crc.log
for i in 1 2; do
  timeout -k 10 120 python3 tools/c4_crc_probe.py > gpurun_out/r6c/c4_lds12_$i.txt 2>&1 && \
  CFSEC_CRC_LDS12=0 timeout -k 10 120 python3 tools/c4_crc_probe.py > gpurun_out/r6c/c4_vperm_$i.txt 2>&1 || exit $?
done
for f in gpurun_out/r6c/c4_*.txt; do echo "== $f"; grep "us per call\|blobs" $f; done
