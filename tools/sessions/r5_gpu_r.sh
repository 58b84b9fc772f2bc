# round-5 session R: register-table fixed-K kernels -- the C4 local probes, then the full GPU suite + smoke
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 120 tools/c4l_pattern_probe > gpurun_out/r5/c4l_pattern3.txt 2>&1 || exit $?
head -4 gpurun_out/r5/c4l_pattern3.txt
timeout -k 10 120 python3 tools/c4_local_probe.py > gpurun_out/r5/c4l_regtab.txt 2>&1 || exit $?
cat gpurun_out/r5/c4l_regtab.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r5/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/r5/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' 2>&1 | tail -2
