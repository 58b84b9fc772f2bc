# Round 6, session E: full GPU suite + smoke on the current library (C4's lookup-kernel fused encode +
# 18 checksums as default, pinned host-range registry, cfsec_stream_copy), the C-ABI segment latency
# tool on HBM / page-locked / pageable shards, then one bench run (new fields: stream_copy_GBps,
# pcie_peaks, *_cabi_us for host memory).
set -o pipefail
mkdir -p gpurun_out/r6e
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r6e/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r6e/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r6e/pytest_gpu.log
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' 2>&1 | tail -1
timeout -k 10 120 ./tools/seg_latency 200 null > gpurun_out/r6e/seg_latency_null.json 2>&1 && \
timeout -k 10 120 ./tools/seg_latency 200 > gpurun_out/r6e/seg_latency_own.json 2>&1 || exit $?
cat gpurun_out/r6e/seg_latency_null.json
CFSEC_HOST_TIMING=1 timeout -k 10 120 ./tools/seg_latency 20 null > gpurun_out/r6e/seg_latency_phases.txt 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > gpurun_out/r6e/bench.json 2> gpurun_out/r6e/bench.err || { tail -20 gpurun_out/r6e/bench.err; exit 1; }
tail -c 300 gpurun_out/r6e/bench.json
