# round-5 session F: NULL-stream single calls (Go's nil stream) and the C4 / C5 synchronous batch
# calls' host phases
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 120 ./tools/seg_latency 300 null > gpurun_out/r5/seg_latency_null.json 2>&1 && \
CFSEC_HOST_TIMING=1 timeout -k 10 120 ./tools/seg_latency 10 null > /dev/null 2> gpurun_out/r5/seg_latency_null_phases.err && \
CFSEC_HOST_TIMING=1 timeout -k 10 300 python3 tools/host_timing.py > gpurun_out/r5/host_timing.txt 2> gpurun_out/r5/host_timing.err
rc=$?
cat gpurun_out/r5/seg_latency_null.json gpurun_out/r5/host_timing.txt
tail -8 gpurun_out/r5/seg_latency_null_phases.err
grep -A12 -- '--- C4 local' gpurun_out/r5/host_timing.err | tail -13
exit $rc
