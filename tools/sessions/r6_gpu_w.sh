# Round 6, session W: the 16 + 20 code's output rows' Horner registers in LDS too (no spilled VGPRs):
# parity tests, the shape sweep against the build that keeps them in registers (33 spilled).
set -o pipefail
mkdir -p gpurun_out/r6w
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu tests/test_gpu_bs_crc_fused.py \
  > gpurun_out/r6w/pytest_bs_crc.log 2>&1 || { tail -40 gpurun_out/r6w/pytest_bs_crc.log; exit 1; }
tail -1 gpurun_out/r6w/pytest_bs_crc.log
for v in base lo0 base lo0; do
  b=./tools/gf_shapes; [ $v = base ] || b=probes_bin/$v/gf_shapes
  echo "== $v" >> gpurun_out/r6w/shapes.txt
  timeout -k 10 200 $b >> gpurun_out/r6w/shapes.txt 2>&1 || exit $?
done
grep -E "==|EC16P20 global|EC16P20L2 fused|EC6P10L2 fused" gpurun_out/r6w/shapes.txt
exit 0
