# Round 4: the multi-GPU repair (Reconstruct + Verify on column slices) on the GPU, then the bench's
# configs[4] leg at N = 1 and rehearsed at N = 2 (gloo, both ranks on the box's one GPU).
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_repair_dist.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r4_repair_tests.log 2>&1
timeout -k 10 300 python -u bench.py --steps 6 --warmup 2 --no-cpu --no-pmc --op-seconds 0.3 > gpurun_out/r4_bench_n1.json 2> gpurun_out/r4_bench_n1.err
CFSEC_BENCH_SHARE_DEVICE=1 CFSEC_BENCH_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 6 --warmup 2 --no-cpu --no-pmc --op-seconds 0.3 > gpurun_out/r4_bench_n2.json 2> gpurun_out/r4_bench_n2.err
