# Round-3 probe (variants reverted after it: no gain): the standalone CRC pass (crc32.hip) with all 16 tiles of a workgroup's run in flight
# (CFSEC_CRC_AHEAD=16), the epilogue basis loaded before the fold (CFSEC_CRC_BASIS_EARLY=1), both;
# C5's tasklet with / without checksums, and gf_shapes' crc-only column (the long-row case).
set -e
mkdir -p gpurun_out
for v in base a16 early a16early base a16 early a16early; do
  lib=chubaofs_amd/libcfsec.so; [ $v = base ] || lib=probes_bin/$v/libcfsec.so
  echo "== $v" >> gpurun_out/crc_pass_ab.txt
  CFSEC_LIB_PATH=$lib C5_REPS=100 timeout -k 10 200 python tools/c5_crc_probe.py 2>&1 | grep crcs >> gpurun_out/crc_pass_ab.txt
done
for v in base a16 early a16early; do
  b=tools/gf_shapes; [ $v = base ] || b=probes_bin/$v/gf_shapes
  echo "== $v sweep" >> gpurun_out/crc_pass_ab.txt
  timeout -k 10 150 $b | grep -E "shape|EC12P4|EC16P20L2 repair" >> gpurun_out/crc_pass_ab.txt
done
