# Round 6, session BC: paired strided tiles with the shifted plane tables built on the host once per
# stride (cached on the device) -- the fused-route and tail tests, then the shape sweep and put-batch
# probes with CFSEC_BC_PAIR=0 / 1 (same library), alternated.
set -o pipefail
mkdir -p gpurun_out/r6bc
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bs_crc_fused.py \
  tests/test_gpu_bs_crc_tail.py > gpurun_out/r6bc/pytest.log 2>&1 || { tail -40 gpurun_out/r6bc/pytest.log; exit 1; }
tail -1 gpurun_out/r6bc/pytest.log
for v in 0 1 0 1; do
  echo "== CFSEC_BC_PAIR=$v" >> gpurun_out/r6bc/shapes.txt
  CFSEC_BC_PAIR=$v timeout -k 10 200 ./tools/gf_shapes > gpurun_out/r6bc/shapes_$v.txt 2>&1 || exit $?
  grep -E "EC12P4|EC6P6|EC6P10L2 fused|EC16P20L2 fused|EC16P20 global|EC12P9|EC6P8|EC3P3|EC4P4" gpurun_out/r6bc/shapes_$v.txt | awk '{print $1,$2,$3,$4,$(NF-3)}' >> gpurun_out/r6bc/shapes.txt
  echo "== CFSEC_BC_PAIR=$v" >> gpurun_out/r6bc/probe.txt
  for m in "EC6P10L2 699051 48" "EC12P4 5592406 8" "EC6P6 174763 256"; do
    set -- $m
    CFSEC_BC_PAIR=$v timeout -k 10 120 python tools/lrc_crc_probe.py $1 $2 $3 >> gpurun_out/r6bc/probe.txt 2>&1 || { cat gpurun_out/r6bc/probe.txt; exit 1; }
  done
done
cat gpurun_out/r6bc/shapes.txt
grep -v amdgpu.ids gpurun_out/r6bc/probe.txt | grep -E "==|crcs=True|all"
exit 0
