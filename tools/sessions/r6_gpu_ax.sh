# Round 6, session AX: crc32block's resident-grid launch with the whole resident grid (CFSEC_BLK_GRID=1,
# the remainder blocks one more per workgroup) against as few workgroups as give equal counts (0):
# the crc32block GPU tests, then the bench's crc32block legs, alternated.
set -o pipefail
mkdir -p gpurun_out/r6ax
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ -k "crc32block or block" \
  > gpurun_out/r6ax/pytest.log 2>&1 || { tail -40 gpurun_out/r6ax/pytest.log; exit 1; }
tail -1 gpurun_out/r6ax/pytest.log
for v in 0 1 0 1; do
  CFSEC_BLK_GRID=$v timeout -k 10 300 python bench.py --no-cpu --no-pmc > gpurun_out/r6ax/bench_$v.json 2> gpurun_out/r6ax/bench_$v.err || exit $?
  python3 - "$v" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/r6ax/bench_{sys.argv[1]}.json"))
print("grid", sys.argv[1], "blk enc", d["crc32block_encode_roofline_frac"], "dec", d["crc32block_decode_roofline_frac"], "value", d["value"])
PY
done
exit 0
