# round-5 session W: clamped row ends in the fixed-K kernels -- ragged-end tests first, C4 local probes,
# the shape sweep, the full GPU suite + smoke
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "ragged or fixed_kernel_output or reconstruct" > gpurun_out/r5/pytest_ragged.log 2>&1; rc=$?
tail -3 gpurun_out/r5/pytest_ragged.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tools/c4l_pattern_probe > gpurun_out/r5/c4l_pattern5.txt 2>&1 || exit $?
sed -n 1,6p gpurun_out/r5/c4l_pattern5.txt
timeout -k 10 120 python3 tools/c4_local_probe.py > gpurun_out/r5/c4l_regtab3.txt 2>&1 || exit $?
cat gpurun_out/r5/c4l_regtab3.txt
timeout -k 10 200 ./tools/gf_shapes > gpurun_out/r5/shape_sweep_w.txt 2>&1 || exit $?
cat gpurun_out/r5/shape_sweep_w.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r5/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r5/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' 2>&1 | tail -1
