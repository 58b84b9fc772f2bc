# round-5 session G: hipStreamQuery(NULL) against a blocking stream's pending work, then the
# NULL-stream single call with the idle-null-stream fast path
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 60 ./tools/null_query_probe > gpurun_out/r5/null_query_probe.txt 2>&1 && \
timeout -k 10 120 ./tools/seg_latency 300 null > gpurun_out/r5/seg_latency_null2.json 2>&1 && \
timeout -k 10 120 ./tools/seg_latency 300 > gpurun_out/r5/seg_latency2.json 2>&1
rc=$?
cat gpurun_out/r5/null_query_probe.txt gpurun_out/r5/seg_latency_null2.json gpurun_out/r5/seg_latency2.json
exit $rc
