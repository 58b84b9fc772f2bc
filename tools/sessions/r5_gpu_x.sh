# round-5 session X: clamped row ends in the lookup-product kernels -- sweep, then the full GPU suite + smoke
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 200 ./tools/gf_shapes > gpurun_out/r5/shape_sweep_x.txt 2>&1 || exit $?
cat gpurun_out/r5/shape_sweep_x.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r5/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r5/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' 2>&1 | tail -1
