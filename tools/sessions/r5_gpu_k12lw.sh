# round-5: the k = 12 lookup kernel with 8-byte lane chunks (probes_bin/r5_k12lw2, CFSEC_LUT_K12_LW=2:
# EC12P9's Verify then takes the early compare loads) -- its GPU tests, then the shape sweep
# alternated with the shipped library
set -o pipefail
mkdir -p gpurun_out/r5k
CFSEC_LIB_PATH=probes_bin/r5_k12lw2/libcfsec.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r5k/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/r5k/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 ./tools/gf_shapes > gpurun_out/r5k/base_$i.txt 2>&1 || exit $?
  timeout -k 10 200 ./probes_bin/r5_k12lw2/gf_shapes > gpurun_out/r5k/lw2_$i.txt 2>&1 || exit $?
done
exit 0
