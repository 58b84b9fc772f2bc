# Round 4: field-form 16x16-dyadic kernels (gf_dyadic16f.hpp) -- correctness on the GPU tests that
# reach them, then the A/B against the byte-form kernels (CFSEC_DY16F=0): C5's tasklet (c5_crc_probe)
# and the shape sweep.
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_lrc_oracle.py tests/test_gpu_batch.py tests/test_gpu_ec.py tests/test_gpu_cabi.py tests/test_repair_dist.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_dy16f_tests.log 2>&1
for v in 0 1 0 1; do
  echo "CFSEC_DY16F=$v" >> gpurun_out/r4_dy16f_ab.txt
  CFSEC_DY16F=$v C5_REPS=50 timeout -k 10 120 python3 tools/c5_crc_probe.py >> gpurun_out/r4_dy16f_ab.txt 2>&1
done
for v in 0 1; do
  echo "CFSEC_DY16F=$v" >> gpurun_out/r4_dy16f_shapes.txt
  CFSEC_DY16F=$v timeout -k 10 180 tools/gf_shapes >> gpurun_out/r4_dy16f_shapes.txt 2>&1
done
