# Round 6, session BE: EC3P3 / EC4P4's fused encode + checksums with up to 8 waves per SIMD
# (CFSEC_BC_WMAX=8: EC3P3 at 5) against the shipped cap of 4 -- shape sweep and put-batch probe, alternated.
set -o pipefail
mkdir -p gpurun_out/r6be
export TMPDIR=/tmp
for v in main wmax8 main wmax8; do
  if [ $v = main ]; then sh=tools/gf_shapes; lib=$PWD/chubaofs_amd/libcfsec.so; else sh=probes_bin/bc_$v/gf_shapes; lib=$PWD/probes_bin/bc_$v/libcfsec.so; fi
  echo "== $v" >> gpurun_out/r6be/shapes.txt
  timeout -k 10 200 $sh > gpurun_out/r6be/shapes_$v.txt 2>&1 || exit $?
  grep -E "EC3P3|EC4P4" gpurun_out/r6be/shapes_$v.txt | awk '{print $1,$2,$3,$4,$(NF-3)}' >> gpurun_out/r6be/shapes.txt
  echo "== $v" >> gpurun_out/r6be/probe.txt
  CFSEC_LIB_PATH=$lib timeout -k 10 120 python tools/lrc_crc_probe.py EC3P3 1398102 16 >> gpurun_out/r6be/probe.txt 2>&1 || { cat gpurun_out/r6be/probe.txt; exit 1; }
done
cat gpurun_out/r6be/shapes.txt
grep -v amdgpu.ids gpurun_out/r6be/probe.txt | grep -E "==|crcs=True|all"
exit 0
