# The LRC fused encode (EC16P20L2) through the ec seam with and without the bit-sliced kernel: wall
# time per call, parity checksum (equal in both runs), and the kernel trace of each run.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r4_bs16_lrc.txt
: > $out
for v in 1 0 1 0; do
  echo "== CFSEC_BS16=$v" >> $out
  CFSEC_BS16=$v timeout -k 10 120 python tools/bs16_lrc_check.py >> $out 2>&1
done
for v in 1 0; do
  CFSEC_BS16=$v timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bs16lrc$v -o run -- python3 tools/bs16_lrc_check.py > /dev/null 2>&1
  echo "== kernels, CFSEC_BS16=$v" >> $out
  grep -h "bs16\|dy16" gpurun_out/bs16lrc$v/run_kernel_stats.csv | cut -c1-160 >> $out || true
done
cat $out
