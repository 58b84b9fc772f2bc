# N = 2 shared-GPU rehearsal (gloo) of the bench, first with the round-4 kernels (no exit drain,
# debug flag words), then with the shipped library.  Exit 3 = a secondary gate failed (a result).
set -o pipefail
mkdir -p gpurun_out/r5
CFSEC_LIB_PATH=probes_bin/r5_nodrain_dbg/libcfsec.so CFSEC_BENCH_SHARE_DEVICE=1 CFSEC_BENCH_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --no-cpu --no-pmc --op-seconds 0.5 > gpurun_out/r5/bench_n2_nodrain.json 2> gpurun_out/r5/bench_n2_nodrain.err
rc=$?; echo "nodrain rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 3 ] || exit $rc
CFSEC_BENCH_SHARE_DEVICE=1 CFSEC_BENCH_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --no-cpu --no-pmc --op-seconds 0.5 > gpurun_out/r5/bench_n2.json 2> gpurun_out/r5/bench_n2.err
rc=$?; echo "shipped rc=$rc"
grep -h 'gate(s) failed\|AssertionError' gpurun_out/r5/bench_n2_nodrain.err gpurun_out/r5/bench_n2.err
exit $rc
