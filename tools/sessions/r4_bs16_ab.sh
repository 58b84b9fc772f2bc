# A/B of the bit-sliced EC16P20(L2) encode (gf_bs16.hip) against the dyadic kernel, alternating
# runs of tools/gf_shapes on one box, plus a kernel trace of one run to show which kernel ran.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r4_bs16_ab.txt
: > $out
for i in 1 2 3; do
  for v in 1 0; do
    echo "== CFSEC_BS16=$v run $i" >> $out
    CFSEC_BS16=$v timeout -k 10 120 tools/gf_shapes 2>&1 | grep -E "EC16P20 global|EC16P20L2 fused" >> $out
  done
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bs16prof -o run -- tools/gf_shapes > /dev/null 2>&1
grep -h "bs16\|gf_dy16_kernel" gpurun_out/bs16prof/run_kernel_stats.csv | cut -c1-200 >> $out || true
cat $out
