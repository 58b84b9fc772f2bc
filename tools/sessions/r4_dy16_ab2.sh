# Round 4: 16x16-dyadic repair forms on C5's tasklet (c5_crc_probe, per-call device time):
# CFSEC_DY16F=0 round-3 byte form, 2 byte form with slot-ordered inputs (default), 1 field form
# (W = 1), and the field form at W = 2 (probes_bin/f2); then VALU instruction counts per form.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_batch.py tests/test_gpu_lrc_oracle.py tests/test_repair_dist.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4_dy16_tests.log 2>&1
out=gpurun_out/r4_dy16_ab2.txt
for rep in 1 2; do
  for v in 0 2 1; do
    echo "CFSEC_DY16F=$v" >> $out
    CFSEC_DY16F=$v C5_REPS=50 timeout -k 10 120 python3 tools/c5_crc_probe.py >> $out 2>&1
  done
  echo "CFSEC_DY16F=1 W=2 (probes_bin/f2)" >> $out
  CFSEC_LIB_PATH=probes_bin/f2/libcfsec.so CFSEC_DY16F=1 C5_REPS=50 timeout -k 10 120 python3 tools/c5_crc_probe.py >> $out 2>&1
done
for v in 0 2; do
  echo "CFSEC_DY16F=$v" >> gpurun_out/r4_dy16_shapes.txt
  CFSEC_DY16F=$v timeout -k 10 180 tools/gf_shapes >> gpurun_out/r4_dy16_shapes.txt 2>&1
done
export TMPDIR=/tmp C5_REPS=5
for v in 0 2; do
  CFSEC_DY16F=$v timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_dy16_$v -o run --output-format csv -- python3 tools/c5_crc_probe.py > gpurun_out/pmc_dy16_$v.log 2>&1
  python3 tools/pmc_summary.py gpurun_out/pmc_dy16_$v > gpurun_out/pmc_dy16_$v.txt
done
