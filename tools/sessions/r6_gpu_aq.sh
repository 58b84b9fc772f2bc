# Round 6, session AQ: the bit-sliced fused kernel's lane fold padded to the next power of two of its
# row count (8 / 16 / 32 / 64; was 32 or 64) -- the fused-route and tail-wave tests, then the shape
# sweep and put-batch probes against the 32-row padding (probes_bin/bc_np32), alternated.
set -o pipefail
mkdir -p gpurun_out/r6aq
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bs_crc_fused.py \
  tests/test_gpu_bs_crc_tail.py > gpurun_out/r6aq/pytest.log 2>&1 || { tail -40 gpurun_out/r6aq/pytest.log; exit 1; }
tail -1 gpurun_out/r6aq/pytest.log
for v in np32 new np32 new; do
  if [ $v = np32 ]; then sh=probes_bin/bc_np32/gf_shapes; lib=$PWD/probes_bin/bc_np32/libcfsec.so; else sh=tools/gf_shapes; lib=$PWD/chubaofs_amd/libcfsec.so; fi
  echo "== $v" >> gpurun_out/r6aq/shapes.txt
  timeout -k 10 200 $sh > gpurun_out/r6aq/shapes_$v.txt 2>&1 || exit $?
  grep -E "EC12P4|EC6P6|EC3P3|EC4P4|EC10P4|EC6P8|EC6P3 |EC16P4" gpurun_out/r6aq/shapes_$v.txt | cut -c1-150 >> gpurun_out/r6aq/shapes.txt
  echo "== $v" >> gpurun_out/r6aq/probe.txt
  for m in "EC12P4 699051 24" "EC3P3 1398102 16"; do
    set -- $m
    CFSEC_LIB_PATH=$lib timeout -k 10 120 python tools/lrc_crc_probe.py $1 $2 $3 >> gpurun_out/r6aq/probe.txt 2>&1 || { cat gpurun_out/r6aq/probe.txt; exit 1; }
  done
done
cat gpurun_out/r6aq/shapes.txt
grep -v amdgpu.ids gpurun_out/r6aq/probe.txt | grep -E "==|crcs=True|all"
exit 0
