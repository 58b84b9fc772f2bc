# A/B of the fused encode+CRC kernels (round 3): the v_perm product kernel (CFSEC_CRC_LDS=0) against
# the lookup-product kernel (CFSEC_CRC_LDS=1, m <= 4), x workgroups per launch (CFSEC_CRC_GROUPS).
# Parity first: the fused-CRC GPU tests under the lookup kernel.  Every GPU step has its own limit.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
[ -n "$AB_SKIP_TESTS" ] || CFSEC_CRC_LDS=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_crc.py tests/test_gpu_batch.py tests/test_gpu_ec.py \
  -k "crc or Crc or CRC" -x -q --timeout 120 --timeout-method thread > gpurun_out/lds_tests.log 2>&1
[ -n "$AB_SKIP_TESTS" ] || tail -2 gpurun_out/lds_tests.log
for v in ${AB_VARIANTS:-0:1024 1:1024 0:768 1:768 1:512 1:1536}; do
  lds=${v%%:*}; g=${v##*:}
  echo "== lds=$lds groups=$g" >> gpurun_out/crc_lds_ab.txt
  CFSEC_CRC_LDS=$lds CFSEC_CRC_GROUPS=$g timeout -k 10 120 tools/gf_shapes >> gpurun_out/crc_lds_ab.txt
done
cat gpurun_out/crc_lds_ab.txt | awk '{print $1,$2,$3,$4,$5,$6,$14,$15,$16,$17}'
