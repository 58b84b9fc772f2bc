# Round-3 probe: virtual-group (512-thread) variants of the lookup-product fused CRC kernel, then PMC
# passes of the lookup kernel (lds_d4) against the v_perm kernel.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in v2w4d6 v2w6d2 v2w4d4 lds_d4; do
  for g in 768 1024; do
    echo "== $v lds=1 groups=$g" >> gpurun_out/crc_lds_ab3.txt
    CFSEC_CRC_LDS=1 CFSEC_CRC_GROUPS=$g timeout -k 10 120 probes_bin/$v/gf_shapes >> gpurun_out/crc_lds_ab3.txt
  done
done
mkdir -p probes_bin/perm && cp tools/gf_shapes probes_bin/perm/gf_shapes
CFSEC_CRC_LDS=1 CFSEC_CRC_GROUPS=768 bash tools/pmc_ab.sh probes_bin/lds_d4/gf_shapes
CFSEC_CRC_LDS=0 bash tools/pmc_ab.sh probes_bin/perm/gf_shapes
