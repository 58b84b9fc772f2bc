# round-5: the scattered C5 false Verify flag -- N = 2 shared-GPU rehearsals alternating the shipped
# library and a diagnosis build whose bit-sliced kernels copy rows into LDS through registers instead
# of LDS-DMA (CFSEC_BS_NODMA=1); each rehearsal's gate failures listed
set -o pipefail
mkdir -p gpurun_out/r5n
CFSEC_LIB_PATH=probes_bin/r5_nodma/libcfsec.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bs_crc.py tests/test_gpu_concurrency.py > gpurun_out/r5n/pytest_nodma.log 2>&1; rc=$?
tail -1 gpurun_out/r5n/pytest_nodma.log
[ $rc -eq 0 ] || exit $rc
CFSEC_LIB_PATH=probes_bin/r5_nodma/libcfsec.so C5_REPS=30 timeout -k 10 120 python3 tools/c5_scatter_probe.py 2>&1 | grep -v amdgpu.ids
for i in 1 2 3; do
  for v in base nodma; do
    if [ $v = nodma ]; then export CFSEC_LIB_PATH=probes_bin/r5_nodma/libcfsec.so; else unset CFSEC_LIB_PATH; fi
    CFSEC_BENCH_SHARE_DEVICE=1 CFSEC_BENCH_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --no-cpu --no-pmc --op-seconds 0.5 > gpurun_out/r5n/n2_${v}_$i.json 2> gpurun_out/r5n/n2_${v}_$i.err; rc=$?
    python3 -c "import json; d=json.loads(open('gpurun_out/r5n/n2_${v}_$i.json').read().strip().splitlines()[-1]); print('$v $i rc=$rc', d.get('gate_failures'), d['configs']['C5_EC16P20L2_repair_tasklet'].get('scattered_kernel_ms'))" || echo "$v $i rc=$rc (no line)"
    [ $rc -eq 0 ] || [ $rc -eq 3 ] || exit $rc
  done
done
unset CFSEC_LIB_PATH
