# Round-3 probe: the 16x16-dyadic kernels' output stores non-temporal (shipped) vs plain, on C5's
# tasklet with / without the rebuilt shards' checksums (the CRC pass re-reads the stored rows) and
# on EC16P20(L2) in the shape sweep.
set -e
mkdir -p gpurun_out
for v in base plainst base plainst; do
  lib=chubaofs_amd/libcfsec.so; [ $v = base ] || lib=probes_bin/$v/libcfsec.so
  echo "== $v" >> gpurun_out/dy16_st_ab.txt
  CFSEC_LIB_PATH=$lib timeout -k 10 200 python tools/c5_crc_probe.py >> gpurun_out/dy16_st_ab.txt 2>&1
done
for v in base plainst; do
  b=tools/gf_shapes; [ $v = base ] || b=probes_bin/$v/gf_shapes
  echo "== $v sweep" >> gpurun_out/dy16_st_ab.txt
  timeout -k 10 150 $b | grep -E "shape|EC16P20" >> gpurun_out/dy16_st_ab.txt
done
