# full GPU test suite + smoke (round 5)
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r5/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/r5/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' 2>&1 | tail -2
