# Round-3 probe: lookup pipelining depth (CFSEC_LDS_PIPE) x virtual groups, lookup fused CRC kernel.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in p2 p0 p1 p3 v2p1 v2p2 p2; do
  b=tools/gf_shapes; [ $v = p2 ] || b=probes_bin/$v/gf_shapes
  for g in ${AB_GROUPS:-768 1024}; do
    echo "== $v lds=1 groups=$g" >> gpurun_out/crc_lds_ab4.txt
    CFSEC_CRC_LDS=1 CFSEC_CRC_GROUPS=$g timeout -k 10 120 $b >> gpurun_out/crc_lds_ab4.txt
  done
done
