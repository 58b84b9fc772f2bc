# round-5: the scattered C5 false Verify flag -- N = 2 rehearsals with the row offsets in the kernel
# argument block (CFSEC_BS_DTAB=0: ~20 bids per launch, no table memory at all)
set -o pipefail
mkdir -p gpurun_out/r5n
export CFSEC_LIB_PATH=probes_bin/r5_dtab0/libcfsec.so
for i in 1 2 3; do
  CFSEC_BENCH_SHARE_DEVICE=1 CFSEC_BENCH_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --no-cpu --no-pmc --op-seconds 0.5 > gpurun_out/r5n/n2_dtab0_$i.json 2> gpurun_out/r5n/n2_dtab0_$i.err; rc=$?
  python3 -c "import json; d=json.loads(open('gpurun_out/r5n/n2_dtab0_$i.json').read().strip().splitlines()[-1]); print('dtab0 $i rc=$rc', d.get('gate_failures'))" || echo "dtab0 $i rc=$rc (no line)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || [ $rc -eq 3 ] || exit $rc
done
