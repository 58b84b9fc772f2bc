# Bisect round 4's false ErrVerify: the N = 2 shared-GPU rehearsal with the exact round-4 library,
# then round 4 + the exit drain only.  Exit 3 from bench = a secondary gate failed (a result).
set -o pipefail
mkdir -p gpurun_out/r5
for v in r4_exact r4_drain; do
  CFSEC_LIB_PATH=probes_bin/$v/libcfsec.so CFSEC_BENCH_SHARE_DEVICE=1 CFSEC_BENCH_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --no-cpu --no-pmc --op-seconds 0.5 > gpurun_out/r5/bench_n2_$v.json 2> gpurun_out/r5/bench_n2_$v.err
  rc=$?; echo "$v rc=$rc"
  grep -h 'gate(s) failed' gpurun_out/r5/bench_n2_$v.err
  [ $rc -eq 0 ] || [ $rc -eq 3 ] || exit $rc
done
