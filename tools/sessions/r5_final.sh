# round-5 final session: GPU suite + smoke on the shipped library, then the bench session (line, trace
# profile, sweep, N = 2 rehearsal)
set -o pipefail
mkdir -p gpurun_out/r5f
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r5f/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/r5f/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' 2>&1 | tail -1
sed 's#gpurun_out/r5c#gpurun_out/r5f#g' tools/r5_bench.sh > /tmp/r5f_bench.sh && bash /tmp/r5f_bench.sh
