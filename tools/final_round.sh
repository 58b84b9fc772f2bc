bash tools/gpu_round.sh && CFSEC_HOST_TIMING=1 timeout -k 10 200 python tools/host_timing.py > gpurun_out/ht.out 2> gpurun_out/ht.err && cat gpurun_out/ht.out
