# The bit-sliced repair (gf_bs16.hip, syndrome form) in the library: GPU tests, then C5's tasklet
# (tools/c5_crc_probe.py) under a kernel trace with the bit-sliced route on and off.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_bsrep.log 2>&1
tail -2 gpurun_out/pytest_bsrep.log
out=gpurun_out/r4_bs16_rep.txt
: > $out
for v in 1 0 1 0; do
  echo "== CFSEC_BS16=$v" >> $out
  CFSEC_BS16=$v timeout -k 10 200 python tools/c5_crc_probe.py >> $out 2>&1
done
for v in 1 0; do
  CFSEC_BS16=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/bsrep$v -o run -- python3 tools/c5_crc_probe.py > /dev/null 2>&1
  echo "== kernels, CFSEC_BS16=$v" >> $out
  grep -h "bs16\|dy16\|crc32" gpurun_out/bsrep$v/run_kernel_stats.csv | cut -c1-170 >> $out || true
done
grep -v amdgpu.ids $out
