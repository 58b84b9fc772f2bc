# Round 6, session BA: the bit-sliced fused kernel at 2 waves per SIMD for the shapes that run 3
# (CFSEC_BC_WPE=2: C4, EC12P4, EC6P6, ...) now that the remainder tiles are tail waves -- shape sweep, alternated.
set -o pipefail
mkdir -p gpurun_out/r6ba
export TMPDIR=/tmp
for v in main wpe2 main wpe2; do
  if [ $v = main ]; then sh=tools/gf_shapes; else sh=probes_bin/bc_$v/gf_shapes; fi
  echo "== $v" >> gpurun_out/r6ba/shapes.txt
  timeout -k 10 200 $sh > gpurun_out/r6ba/shapes_$v.txt 2>&1 || exit $?
  grep -E "EC12P4|EC6P6|EC6P10L2 fused|EC6P10 global|EC6P8|EC10P4|EC4P4|EC3P3" gpurun_out/r6ba/shapes_$v.txt | awk '{print $1,$2,$3,$4,$(NF-3)}' >> gpurun_out/r6ba/shapes.txt
done
cat gpurun_out/r6ba/shapes.txt
exit 0
