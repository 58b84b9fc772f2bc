# round-5 session L: C5 tasklet with / without checksums vs the rebuilt rows' store policy (nt / plain)
# and the checksum pass's load policy (nt / plain)
set -o pipefail
mkdir -p gpurun_out/r5
out=gpurun_out/r5/c5_cache_policy.txt
for i in 1 2; do
  for v in base st1 ld0 st1ld0; do
    echo "== $v ($i)" >> $out
    if [ $v = base ]; then
      C5_REPS=50 timeout -k 10 120 python3 tools/c5_crc_probe.py >> $out 2>&1 || exit $?
    else
      CFSEC_LIB_PATH=probes_bin/r5_$v/libcfsec.so C5_REPS=50 timeout -k 10 120 python3 tools/c5_crc_probe.py >> $out 2>&1 || exit $?
    fi
  done
done
cat $out
timeout -k 10 60 tools/seg_latency 300 > gpurun_out/r5/seg_floor.txt 2>&1 || exit $?; cat gpurun_out/r5/seg_floor.txt
