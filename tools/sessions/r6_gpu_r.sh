# Round 6, session R: the shipped form of the bit-sliced fused encode + checksums (per-row Horner
# registers, W waves per stripe, tree fold; EC6P10L2's route on, EC12P4's off): its tests, the checksum
# suites, C4's put batch against the lookup-product kernel, the shape sweep.
set -o pipefail
mkdir -p gpurun_out/r6r
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bs_crc_fused.py \
  tests/test_gpu_crc.py tests/test_gpu_batch.py > gpurun_out/r6r/pytest.log 2>&1 || { tail -40 gpurun_out/r6r/pytest.log; exit 1; }
tail -1 gpurun_out/r6r/pytest.log
for v in 1 0; do
  echo "== CFSEC_BS_CRC=$v" >> gpurun_out/r6r/c4.txt
  CFSEC_BS_CRC=$v timeout -k 10 120 python tools/c4_crc_probe.py >> gpurun_out/r6r/c4.txt 2>&1 || exit $?
done
grep -E "==|us per call|all" gpurun_out/r6r/c4.txt
timeout -k 10 200 ./tools/gf_shapes > gpurun_out/r6r/shapes.txt 2>&1 || exit $?
grep -E "EC12P4|EC6P10L2 fused" gpurun_out/r6r/shapes.txt
exit 0
