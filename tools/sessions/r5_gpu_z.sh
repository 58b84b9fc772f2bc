# round-5 session Z: the clamped row end in the dyadic and lookup-product kernels (one body) -- the lookup
# diagnosis, the ragged-end and batch tests, the sweep, then the full GPU suite + smoke
set -o pipefail
mkdir -p gpurun_out/r5z3
timeout -k 10 120 python3 tools/lut_clamp_diag.py > gpurun_out/r5z3/lutdiag.txt 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5z3/lutdiag.txt | grep -v ": OK" | grep -v "golden: True" | head -10
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_batch.py > gpurun_out/r5z3/pytest_a.log 2>&1; rc=$?
tail -2 gpurun_out/r5z3/pytest_a.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 ./tools/gf_shapes > gpurun_out/r5z3/shape_sweep.txt 2>&1 || exit $?
cat gpurun_out/r5z3/shape_sweep.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r5z3/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/r5z3/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' 2>&1 | tail -1
