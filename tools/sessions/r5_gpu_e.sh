# round-5 session E: single-call latency itemised (C++ caller, then the Python layers), and the
# engine's phase times of a few calls
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 120 ./tools/seg_latency 300 > gpurun_out/r5/seg_latency.json 2> gpurun_out/r5/seg_latency.err && \
CFSEC_HOST_TIMING=1 timeout -k 10 120 ./tools/seg_latency 20 > /dev/null 2> gpurun_out/r5/seg_latency_phases.err && \
timeout -k 10 180 python3 tools/r5_latency.py > gpurun_out/r5/py_latency.json 2> gpurun_out/r5/py_latency.err
rc=$?
cat gpurun_out/r5/seg_latency.json gpurun_out/r5/py_latency.json
tail -12 gpurun_out/r5/seg_latency_phases.err
exit $rc
