# Round 6, session AU: the bit-sliced fused kernel's strided tiles in pairs (one register jump per pair,
# the earlier tile's terms from plane tables shifted by the stride; CFSEC_BC_PAIR) -- the fused-route and
# tail tests, then the shape sweep and put-batch probes against the unpaired build, alternated.
set -o pipefail
mkdir -p gpurun_out/r6au
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bs_crc_fused.py \
  tests/test_gpu_bs_crc_tail.py > gpurun_out/r6au/pytest.log 2>&1 || { tail -40 gpurun_out/r6au/pytest.log; exit 1; }
tail -1 gpurun_out/r6au/pytest.log
for v in nopair pair nopair pair; do
  if [ $v = nopair ]; then sh=probes_bin/bc_nopair/gf_shapes; lib=$PWD/probes_bin/bc_nopair/libcfsec.so; else sh=tools/gf_shapes; lib=$PWD/chubaofs_amd/libcfsec.so; fi
  echo "== $v" >> gpurun_out/r6au/shapes.txt
  timeout -k 10 200 $sh > gpurun_out/r6au/shapes_$v.txt 2>&1 || exit $?
  grep -E "EC12P4|EC6P6|EC6P10L2 fused|EC16P20L2 fused|EC16P20 global|EC12P9|EC6P8|EC3P3" gpurun_out/r6au/shapes_$v.txt | cut -c1-150 >> gpurun_out/r6au/shapes.txt
  echo "== $v" >> gpurun_out/r6au/probe.txt
  for m in "EC6P10L2 699051 48" "EC12P4 5592406 8" "EC6P6 174763 256"; do
    set -- $m
    CFSEC_LIB_PATH=$lib timeout -k 10 120 python tools/lrc_crc_probe.py $1 $2 $3 >> gpurun_out/r6au/probe.txt 2>&1 || { cat gpurun_out/r6au/probe.txt; exit 1; }
  done
done
grep -E "==|EC" gpurun_out/r6au/shapes.txt | awk 'NF<3{print;next}{print $1,$2,$3,$4,$(NF-3)}'
grep -v amdgpu.ids gpurun_out/r6au/probe.txt | grep -E "==|crcs=True|all"
exit 0
