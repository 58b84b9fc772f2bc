# The bit-sliced encodes for EC15P12 / EC12P9 (and EC16P20(L2)) against the shipped routes:
# GPU tests, then tools/gf_shapes with CFSEC_BS16=1 / 0 alternating.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_bsk.log 2>&1
tail -1 gpurun_out/pytest_bsk.log
out=gpurun_out/r4_bsk_ab.txt
: > $out
for i in 1 2; do
  for v in 1 0; do
    echo "== CFSEC_BS16=$v run $i" >> $out
    CFSEC_BS16=$v timeout -k 10 120 tools/gf_shapes 2>&1 | grep -E "shape|EC16P20 global|EC16P20L2 fused|EC15P12|EC12P9" >> $out
  done
done
cat $out
