# Round 6, session B: the GPU suite on the current library (hazard-free stores, the runtime-k kernel's
# clamped row end, the fused-CRC fallback), then shape sweeps alternated over the current library,
# the current sources with the round-5 stores (C_old) and the two round-5 variants with the new stores
# (A_new, B_new), then one bench run.
set -o pipefail
mkdir -p gpurun_out/r6b
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r6b/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r6b/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r6b/pytest_gpu.log
for i in 1 2; do
  timeout -k 10 200 ./tools/gf_shapes > gpurun_out/r6b/shapes_cur_$i.txt 2>&1 && \
  timeout -k 10 200 ./probes_bin/r6_hz/C_old/gf_shapes > gpurun_out/r6b/shapes_Cold_$i.txt 2>&1 && \
  timeout -k 10 200 ./probes_bin/r6_hz/A_new/gf_shapes > gpurun_out/r6b/shapes_Anew_$i.txt 2>&1 && \
  timeout -k 10 200 ./probes_bin/r6_hz/B_new/gf_shapes > gpurun_out/r6b/shapes_Bnew_$i.txt 2>&1 || exit $?
done
timeout -k 10 400 python -u bench.py > gpurun_out/r6b/bench.json 2> gpurun_out/r6b/bench.err || { tail -20 gpurun_out/r6b/bench.err; exit 1; }
tail -c 600 gpurun_out/r6b/bench.json
