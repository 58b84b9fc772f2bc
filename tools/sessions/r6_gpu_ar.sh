# Round 6, session AR: timing probes of the bit-sliced fused kernel (wrong words, shape sweep only):
# without the Horner registers' jumps (probes_bin/bc_nojump) and without any checksum lookups
# (probes_bin/bc_probe7: product, stores and folds only) against the shipped kernel.
set -o pipefail
mkdir -p gpurun_out/r6ar
export TMPDIR=/tmp
for v in main nojump probe7 main nojump probe7; do
  if [ $v = main ]; then sh=tools/gf_shapes; else sh=probes_bin/bc_$v/gf_shapes; fi
  echo "== $v" >> gpurun_out/r6ar/shapes.txt
  timeout -k 10 200 $sh > gpurun_out/r6ar/shapes_$v.txt 2>&1 || exit $?
  grep -E "EC12P4|EC6P6|EC6P10L2 fused|EC16P20L2 fused" gpurun_out/r6ar/shapes_$v.txt | cut -c1-150 >> gpurun_out/r6ar/shapes.txt
done
grep -E "==|EC12P4|EC6P6|EC6P10L2|EC16P20L2" gpurun_out/r6ar/shapes.txt | awk 'NF<3{print;next}{print $1,$2,$3,$4,$(NF-3)}'
exit 0
