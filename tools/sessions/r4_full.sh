# Round 4 full GPU session: tests, smoke, bench (+ PMC traffic), kernel-trace profile of the bench
# with the timed-region statistics, the N = 2 rehearsal (gloo, both ranks on the box's GPU) and the
# host-side phase timing of the C4 / C5 synchronous calls.
set -e
bash tools/gpu_round.sh
CFSEC_BENCH_SHARE_DEVICE=1 CFSEC_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --no-cpu --no-pmc --op-seconds 0.5 > gpurun_out/bench_n2.json 2> gpurun_out/bench_n2.err
CFSEC_HOST_TIMING=1 timeout -k 10 200 python tools/host_timing.py > gpurun_out/ht.out 2> gpurun_out/ht.err
