# Round 6, session AC: is C4's fused encode + 18 checksums bound by its tiles-per-wave remainder?
# The put batch (48 bids) at row lengths whose 2048-byte tile count per row is 320 (5 per wave at W =
# 64), 321, 342 (the bench's 699,051 B) and 384 (6 per wave): time proportional to the bytes, or to
# the ceiling of tiles per wave.
set -o pipefail
mkdir -p gpurun_out/r6ac
export TMPDIR=/tmp
for S in 655360 657000 699051 786432; do
  echo "== S=$S" >> gpurun_out/r6ac/tail.txt
  timeout -k 10 120 python tools/lrc_crc_probe.py EC6P10L2 $S 48 >> gpurun_out/r6ac/tail.txt 2>&1 || exit $?
done
grep -E "==|us per call|all" gpurun_out/r6ac/tail.txt
exit 0
