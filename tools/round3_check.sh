# Round-3 GPU check: the GPU round (tests, smoke, bench, kernel trace), the shape sweep with and without
# the lookup-product kernels, and the bench line with CFSEC_LUT=0 (A/B of the headline step kernel).
set -e
bash tools/gpu_round.sh
timeout -k 10 120 tools/gf_shapes > gpurun_out/shape_sweep.txt
CFSEC_LUT=0 timeout -k 10 120 tools/gf_shapes > gpurun_out/shape_sweep_nolut.txt
CFSEC_LUT=0 timeout -k 10 300 python bench.py --no-cpu --no-pmc > gpurun_out/bench_nolut.json 2> gpurun_out/bench_nolut.err
