# Round 6, session AG: the host cost of C4's asynchronous batch call (the bench's per-call event pairs
# include the host's enqueue time whenever the host is behind the GPU) -- wall time per call with the
# device held busy, and the library's phase timers for one call.
set -o pipefail
mkdir -p gpurun_out/r6ag
export TMPDIR=/tmp
timeout -k 10 120 python tools/host_call_cost.py EC6P10L2 > gpurun_out/r6ag/host.txt 2>&1 || { cat gpurun_out/r6ag/host.txt; exit 1; }
CFSEC_HOST_TIMING=1 timeout -k 10 120 python tools/host_call_cost.py EC6P10L2 699051 48 > gpurun_out/r6ag/host_timers.txt 2>&1 || exit $?
timeout -k 10 120 python tools/host_call_cost.py EC12P4 5592406 8 >> gpurun_out/r6ag/host.txt 2>&1 || exit $?
cat gpurun_out/r6ag/host.txt
grep cfsec gpurun_out/r6ag/host_timers.txt | sort | uniq -c | sort -rn | head -5
tail -12 gpurun_out/r6ag/host_timers.txt
exit 0
