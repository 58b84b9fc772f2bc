# Round 6, session AN: EC6P6, EC6P3 and EC16P4's encode + checksums on the bit-sliced kernel (the
# first rows of the EC6P10L2 / 16 + 20 networks, CFSEC_BS_CRC bit 6) against their product kernels'
# fused forms -- the put-batch probe (words vs zlib) and the shape sweep, alternated.
set -o pipefail
mkdir -p gpurun_out/r6an
export TMPDIR=/tmp
for v in 55 119 55 119; do
  echo "== CFSEC_BS_CRC=$v" >> gpurun_out/r6an/probe.txt
  for m in "EC6P6 174763 256" "EC6P3 699051 32" "EC16P4 262144 64"; do
    set -- $m
    CFSEC_BS_CRC=$v timeout -k 10 120 python tools/lrc_crc_probe.py $1 $2 $3 >> gpurun_out/r6an/probe.txt 2>&1 || { cat gpurun_out/r6an/probe.txt; exit 1; }
  done
  echo "== CFSEC_BS_CRC=$v" >> gpurun_out/r6an/shapes.txt
  CFSEC_BS_CRC=$v timeout -k 10 200 ./tools/gf_shapes > gpurun_out/r6an/shapes_$v.txt 2>&1 || exit $?
  grep -E "^shape|EC6P6|EC6P3 |EC16P4" gpurun_out/r6an/shapes_$v.txt >> gpurun_out/r6an/shapes.txt
done
grep -v amdgpu.ids gpurun_out/r6an/probe.txt | grep -E "==|crcs=True|all"
cat gpurun_out/r6an/shapes.txt | cut -c1-150
exit 0
