# round-5: lookup-kernel Verify with the compared rows loaded early (now the default) -- the GPU
# tests, then the shape sweep alternated with the CFSEC_LUT_VPRE=0 build (probes_bin/r5_lutvpre0)
set -o pipefail
mkdir -p gpurun_out/r5v
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5v/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/r5v/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 ./tools/gf_shapes > gpurun_out/r5v/on_$i.txt 2>&1 || exit $?
  timeout -k 10 200 ./probes_bin/r5_lutvpre0/gf_shapes > gpurun_out/r5v/off_$i.txt 2>&1 || exit $?
done
exit 0
