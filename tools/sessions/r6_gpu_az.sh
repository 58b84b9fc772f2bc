# Round 6, session AZ: the standalone checksum pass's workgroup total (CFSEC_CRC32_GROUPS_PROBE; 0 = the
# shipped 4096) -- the shape sweep's crc-only column and C5's tasklet with checksums, per value.
set -o pipefail
mkdir -p gpurun_out/r6az
export TMPDIR=/tmp
for v in 0 1792 3584 5376 7168 0; do
  echo "== CFSEC_CRC32_GROUPS_PROBE=$v" >> gpurun_out/r6az/shapes.txt
  CFSEC_CRC32_GROUPS_PROBE=$v timeout -k 10 200 ./tools/gf_shapes > gpurun_out/r6az/shapes_$v.txt 2>&1 || exit $?
  awk 'NR>1{print $1,$2,$3,$4,$NF=="fused"||$NF=="sep"?$(NF-1):$NF}' gpurun_out/r6az/shapes_$v.txt >> gpurun_out/r6az/shapes.txt
  echo "== CFSEC_CRC32_GROUPS_PROBE=$v" >> gpurun_out/r6az/c5.txt
  CFSEC_CRC32_GROUPS_PROBE=$v timeout -k 10 120 python tools/c5_crc_probe.py >> gpurun_out/r6az/c5.txt 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/r6az/c5.txt | grep -E "==|crcs"
exit 0
