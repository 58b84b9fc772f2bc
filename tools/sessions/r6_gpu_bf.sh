# Round 6, session BF: tiles per wave and stripe for the small and mid shapes (CFSEC_BC_TPW: W = ceil(tps / TPW);
# 0 = the shipped W = resident waves / stripes) -- shape sweep, +crc us.
set -o pipefail
mkdir -p gpurun_out/r6bf
export TMPDIR=/tmp
for v in 0 4 8 16 0 4 8 16; do
  echo "== CFSEC_BC_TPW=$v" >> gpurun_out/r6bf/shapes.txt
  CFSEC_BC_TPW=$v timeout -k 10 200 ./tools/gf_shapes > gpurun_out/r6bf/shapes_$v.txt 2>&1 || exit $?
  grep -E "EC12P4|EC6P6|EC6P10L2 fused|EC6P10 global|EC16P20L2 fused|EC12P9|EC15P12|EC10P4|EC6P8|EC4P4|EC3P3|EC16P4" gpurun_out/r6bf/shapes_$v.txt | awk '{print $1,$2,$3,$4,$(NF-3)}' >> gpurun_out/r6bf/shapes.txt
done
exit 0
