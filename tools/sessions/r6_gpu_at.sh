# Round 6, session AT: HBM traffic of the bit-sliced fused encode + checksum kernels (rocprofv3 --pmc,
# FETCH_SIZE and WRITE_SIZE in separate passes) on C4's put batch, EC12P4's 64 MiB blobs and EC6P6's
# 1 MiB blobs (tools/lrc_crc_probe.py), per launch against the algorithmic bytes.
set -o pipefail
mkdir -p gpurun_out/r6at
export TMPDIR=/tmp
for m in "EC6P10L2 699051 48" "EC12P4 5592406 8" "EC6P6 174763 256"; do
  set -- $m
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/r6at/$1_$c -o pmc -- python3 tools/lrc_crc_probe.py $1 $2 $3 \
      > gpurun_out/r6at/$1_$c.log 2>&1 || { tail -20 gpurun_out/r6at/$1_$c.log; exit 1; }
  done
done
python3 tools/pmc_kernel_traffic.py gpurun_out/r6at/EC6P10L2_FETCH_SIZE gpurun_out/r6at/EC6P10L2_WRITE_SIZE BsEc6p10l2=603980064 > gpurun_out/r6at/traffic.txt
python3 tools/pmc_kernel_traffic.py gpurun_out/r6at/EC12P4_FETCH_SIZE gpurun_out/r6at/EC12P4_WRITE_SIZE BsEc12p4=715827968 >> gpurun_out/r6at/traffic.txt
python3 tools/pmc_kernel_traffic.py gpurun_out/r6at/EC6P6_FETCH_SIZE gpurun_out/r6at/EC6P6_WRITE_SIZE "BsEc6p10l2, 6=536871936" >> gpurun_out/r6at/traffic.txt
rm -rf gpurun_out/r6at/*_SIZE
cat gpurun_out/r6at/traffic.txt
exit 0
