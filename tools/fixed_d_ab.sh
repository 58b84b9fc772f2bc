# Round-3 probe: row lookahead of the fixed-K kernels (CFSEC_FIXED_D 2 shipped / 4 / 8), shape sweep, same call.
set -e
mkdir -p gpurun_out
for v in base fixd4 fixd8 base fixd4 fixd8; do
  b=tools/gf_shapes; [ $v = base ] || b=probes_bin/$v/gf_shapes
  echo "== $v" >> gpurun_out/fixed_d_ab.txt
  timeout -k 10 120 $b >> gpurun_out/fixed_d_ab.txt
done
