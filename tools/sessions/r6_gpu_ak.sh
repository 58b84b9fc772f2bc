# Round 6, session AK: the shape sweep's EC12P4 rows (64 MiB and 4 MiB blobs) with EC12P4's bit-sliced
# route off (53), on for rows >= 2 MiB (55) and at every length (63), alternated -- after the tail waves.
set -o pipefail
mkdir -p gpurun_out/r6ak
export TMPDIR=/tmp
for v in 53 55 63 53 55 63; do
  echo "== CFSEC_BS_CRC=$v" >> gpurun_out/r6ak/shapes.txt
  CFSEC_BS_CRC=$v timeout -k 10 200 ./tools/gf_shapes > gpurun_out/r6ak/shapes_$v.txt 2>&1 || exit $?
  grep -E "^shape|EC12P4" gpurun_out/r6ak/shapes_$v.txt >> gpurun_out/r6ak/shapes.txt
done
cat gpurun_out/r6ak/shapes.txt
exit 0
