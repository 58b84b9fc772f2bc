# Round 6, session Q: C4's per-row fused kernel with fewer tiles per wave and stripe (more waves per
# stripe, more stripes per wave, one fold per wave and stripe): CFSEC_BC_TPW A/B on the put batch.
set -o pipefail
mkdir -p gpurun_out/r6q
export TMPDIR=/tmp
for tpw in 0 1 2 3 4; do
  echo "== CFSEC_BC_TPW=$tpw" >> gpurun_out/r6q/c4.txt
  CFSEC_BC_TPW=$tpw CFSEC_BS_CRC=5 timeout -k 10 120 python tools/c4_crc_probe.py >> gpurun_out/r6q/c4.txt 2>&1 || exit $?
done
grep -E "==|us per call|all" gpurun_out/r6q/c4.txt
exit 0
