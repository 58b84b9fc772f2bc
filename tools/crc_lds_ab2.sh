set -e
mkdir -p gpurun_out
for v in lds_d4 lds_d6 lds_d8 base lds_d4; do
  b=tools/gf_shapes; [ $v = base ] || b=probes_bin/$v/gf_shapes
  echo "== $v lds=1 groups=768" >> gpurun_out/crc_lds_ab2.txt
  CFSEC_CRC_LDS=1 CFSEC_CRC_GROUPS=768 timeout -k 10 120 $b >> gpurun_out/crc_lds_ab2.txt
done
