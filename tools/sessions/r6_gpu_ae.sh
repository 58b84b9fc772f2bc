# Round 6, session AE: remainder tiles as tail waves -- C4 with one more whole round moved to the tail
# (CFSEC_BC_TEXTRA=1), and EC6P6L9's plain + checksummed routes with and without, alternated.
set -o pipefail
mkdir -p gpurun_out/r6ae
export TMPDIR=/tmp
for v in "100 0" "100 1" "0 0" "100 0" "100 1"; do
  set -- $v
  echo "== EC6P10L2 CFSEC_BC_TAIL=$1 CFSEC_BC_TEXTRA=$2" >> gpurun_out/r6ae/tail.txt
  CFSEC_BC_TAIL=$1 CFSEC_BC_TEXTRA=$2 timeout -k 10 120 python tools/lrc_crc_probe.py EC6P10L2 699051 48 >> gpurun_out/r6ae/tail.txt 2>&1 || exit $?
done
for v in 0 100 0 100; do
  echo "== EC6P6L9 CFSEC_BC_TAIL=$v" >> gpurun_out/r6ae/tail.txt
  CFSEC_BC_TAIL=$v timeout -k 10 120 python tools/lrc_crc_probe.py EC6P6L9 699051 32 >> gpurun_out/r6ae/tail.txt 2>&1 || exit $?
done
grep -E "==|us per call|all" gpurun_out/r6ae/tail.txt
exit 0
