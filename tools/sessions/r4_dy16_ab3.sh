# Round 4: the 16x16-dyadic repair with the 16x16 block's compared rows loaded before the block
# (CFSEC_DY16_PF=1, default build) vs loaded as each row completes (probes_bin/pf0); C5 tasklet.
set -e
mkdir -p gpurun_out
out=gpurun_out/r4_dy16_ab3.txt
for rep in 1 2; do
  echo "PF=1" >> $out
  C5_REPS=50 timeout -k 10 120 python3 tools/c5_crc_probe.py >> $out 2>&1
  echo "PF=0 (probes_bin/pf0)" >> $out
  CFSEC_LIB_PATH=probes_bin/pf0/libcfsec.so C5_REPS=50 timeout -k 10 120 python3 tools/c5_crc_probe.py >> $out 2>&1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -m gpu -x -q -k "c5 or C5 or EC16P20 or async or crc" --timeout 300 --timeout-method thread > gpurun_out/r4_dy16_tests3.log 2>&1
timeout -k 10 120 tools/c5_pattern_probe > gpurun_out/r4_c5_pattern.txt 2>&1
