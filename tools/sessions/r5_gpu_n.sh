# round-5 session N: launch-call and kernel-argument costs, and the batch calls' launch phases
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 60 tools/seg_latency 300 > gpurun_out/r5/seg_floor2.txt 2>&1 || exit $?
CFSEC_HOST_TIMING=1 timeout -k 10 180 python3 tools/host_timing.py > gpurun_out/r5/host_timing2.txt 2> gpurun_out/r5/host_timing_err2.txt || exit $?
python3 tools/host_phase_summary.py gpurun_out/r5/host_timing_err2.txt > gpurun_out/r5/host_phases2.txt
cat gpurun_out/r5/seg_floor2.txt gpurun_out/r5/host_phases2.txt
