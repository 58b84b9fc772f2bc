# Round 6, session A: the store-data hazard.  The two round-5 "wrong rows" variants with the round-5
# inline-asm stores (old) and with the hazard-free stores (new), each through the parity and batch
# tests; then the shipped library's full GPU suite and smoke.
set -o pipefail
mkdir -p gpurun_out/r6a
for v in A_old A_new B_old B_new; do
  CFSEC_LIB_PATH=$PWD/probes_bin/r6_hz/$v/libcfsec.so timeout -k 10 300 python -u -m pytest -q --timeout 120 \
    --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_batch.py -p no:cacheprovider \
    > gpurun_out/r6a/variant_$v.log 2>&1
  rc=$?
  echo "variant $v rc=$rc: $(tail -1 gpurun_out/r6a/variant_$v.log)"
  # wrong bytes are not faults; anything else (abort, segfault, time limit) ends the session
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r6a/pytest_gpu.log 2>&1
rc=$?
tail -3 gpurun_out/r6a/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' 2>&1 | tail -2
