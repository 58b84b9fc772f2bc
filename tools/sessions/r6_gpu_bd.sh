# Round 6, session BD: the full GPU suite and smoke on the final library (rebuilt after the host-table pairing A/B).
set -o pipefail
mkdir -p gpurun_out/r6bd
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r6bd/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r6bd/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r6bd/pytest_gpu.log
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' 2>&1 | tail -1
exit 0
