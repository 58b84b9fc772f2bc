# round-5 session Y: row-offset tables read from mapped host memory -- scattered tests and probe, then the
# N = 2 shared-GPU rehearsal (where the false Verify flag showed) twice
set -o pipefail
mkdir -p gpurun_out/r5y
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_batch.py tests/test_gpu_bs_crc.py tests/test_gpu_concurrency.py > gpurun_out/r5y/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r5y/pytest.log
[ $rc -eq 0 ] || exit $rc
C5_REPS=50 timeout -k 10 120 python3 tools/c5_scatter_probe.py > gpurun_out/r5y/scatter.txt 2>&1 || exit $?
cat gpurun_out/r5y/scatter.txt
for i in 1 2; do
  CFSEC_BENCH_SHARE_DEVICE=1 CFSEC_BENCH_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --no-cpu --no-pmc --op-seconds 0.5 > gpurun_out/r5y/bench_n2_$i.json 2> gpurun_out/r5y/bench_n2_$i.err; rc=$?
  echo "n2 run $i rc=$rc"
  python3 -c "import json; d=json.loads(open('gpurun_out/r5y/bench_n2_$i.json').read().strip().splitlines()[-1]); print('gate_failures', d.get('gate_failures'), 'scattered', d['configs']['C5_EC16P20L2_repair_tasklet'].get('scattered_kernel_ms'))" || true
  [ $rc -eq 0 ] || exit $rc
done
