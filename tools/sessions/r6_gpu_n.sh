# Round 6, session N: the bit-sliced product's own speed in the fused kernel's structure -- blocked vs
# strided tiles (as gf_bs_kernel), occupancy, register prefetch -- with the checksum lookups removed
# (CFSEC_BC_PROBE=3; timing probes only, wrong words), C4's put batch.
set -o pipefail
mkdir -p gpurun_out/r6n
export TMPDIR=/tmp
for v in pr_probe3_str pr_probe3_str_w4 pr_probe3_str_pf pr_str; do
  echo "== $v" >> gpurun_out/r6n/c4.txt
  CFSEC_LIB_PATH=$PWD/probes_bin/$v/libcfsec.so CFSEC_BS_CRC=5 timeout -k 10 120 python tools/c4_crc_probe.py >> gpurun_out/r6n/c4.txt 2>&1
  rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
grep -E "==|us per call|all" gpurun_out/r6n/c4.txt
exit 0
