# round-5 session M: host phases of the synchronous / asynchronous batch calls (C4, C5)
set -o pipefail
mkdir -p gpurun_out/r5
CFSEC_HOST_TIMING=1 timeout -k 10 180 python3 tools/host_timing.py > gpurun_out/r5/host_timing.txt 2> gpurun_out/r5/host_timing_err.txt || exit $?
timeout -k 10 180 python3 tools/host_timing.py > gpurun_out/r5/host_timing_off.txt 2>&1 || exit $?
python3 tools/host_phase_summary.py gpurun_out/r5/host_timing_err.txt > gpurun_out/r5/host_phases.txt
cat gpurun_out/r5/host_timing.txt gpurun_out/r5/host_timing_off.txt gpurun_out/r5/host_phases.txt
