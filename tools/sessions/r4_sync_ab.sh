# Round 4: synchronous calls end by polling a marker word the stream writes (DeviceContext::finish)
# instead of hipStreamSynchronize -- the GPU tests on it, then the C4 / C5 synchronous call times
# with and without it (CFSEC_SYNC_POLL=0).
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4_sync_tests.log 2>&1
for rep in 1 2; do
  echo "poll" >> gpurun_out/r4_sync_ab.txt
  timeout -k 10 200 python tools/host_timing.py >> gpurun_out/r4_sync_ab.txt 2>/dev/null
  echo "hipStreamSynchronize (CFSEC_SYNC_POLL=0)" >> gpurun_out/r4_sync_ab.txt
  CFSEC_SYNC_POLL=0 timeout -k 10 200 python tools/host_timing.py >> gpurun_out/r4_sync_ab.txt 2>/dev/null
done
