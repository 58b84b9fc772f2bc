# round-5 closing check after the lookup-Verify change: smoke, then the driver's bench line
set -o pipefail
mkdir -p gpurun_out/r5f2
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5f2/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r5f2/smoke.log
timeout -k 10 420 python bench.py > gpurun_out/r5f2/bench.json 2> gpurun_out/r5f2/bench.err || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/r5f2/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['unit'], d['roofline']['frac'], d.get('gate_failures'))"
