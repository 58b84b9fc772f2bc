# Round 4: occupancy of the 16x16-dyadic repair on C5's tasklet: the default (8-byte lanes, 117
# VGPRs, 4 waves/SIMD) vs 4-byte lanes (probes_bin/w1: 71 VGPRs) vs 5 waves forced (probes_bin/wpe5:
# 96 VGPRs + 28 spilled); then the access-pattern ceiling (tools/c5_pattern_probe).
set -e
mkdir -p gpurun_out
out=gpurun_out/r4_dy16_ab4.txt
for rep in 1 2; do
  echo "default" >> $out
  C5_REPS=50 timeout -k 10 120 python3 tools/c5_crc_probe.py >> $out 2>&1
  for v in w1 wpe5; do
    echo "$v" >> $out
    CFSEC_LIB_PATH=probes_bin/$v/libcfsec.so C5_REPS=50 timeout -k 10 120 python3 tools/c5_crc_probe.py >> $out 2>&1
  done
done
timeout -k 10 120 tools/c5_pattern_probe > gpurun_out/r4_c5_pattern.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -m gpu -x -q -k "c5 or C5 or EC16P20 or async or crc" --timeout 300 --timeout-method thread > gpurun_out/r4_dy16_tests4.log 2>&1
