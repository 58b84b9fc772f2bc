# Standalone checksum pass (measured, not shipped): the thread-to-tile-end shift by one mulmod (the probe build) vs the 32-column
# GF(2) basis (probes_bin/crcbasis: UNITS=crc32 tools/build_variant.sh crcbasis -DCFSEC_CRC_MULMOD=0),
# over C5's 256 rebuilt rows and 128 long rows (tools/crc_pass_probe, workgroup-count sweep) and
# C5's tasklet with / without checksums, libraries alternated.
set -e
mkdir -p gpurun_out
out=gpurun_out/r4_crc_mulmod_ab.txt
: > $out
cp chubaofs_amd/libcfsec.so gpurun_out/lib_default.so
for v in default crcbasis default crcbasis; do
  if [ $v = default ]; then cp gpurun_out/lib_default.so chubaofs_amd/libcfsec.so; else cp probes_bin/$v/libcfsec.so chubaofs_amd/libcfsec.so; fi
  echo "== $v" >> $out
  timeout -k 10 120 tools/crc_pass_probe >> $out
  timeout -k 10 200 python tools/c5_crc_probe.py 2>/dev/null | grep -v amdgpu >> $out
done
cp gpurun_out/lib_default.so chubaofs_amd/libcfsec.so
rm -f gpurun_out/lib_default.so
cat $out
