# Round 6, session AP: the bench with C1's new encode + checksum leg (EC6P6 1 MiB blobs through
# cfsec_rs_encode_crc_batch), no CPU legs.
set -o pipefail
mkdir -p gpurun_out/r6ap
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --no-cpu --no-pmc > gpurun_out/r6ap/bench.json 2> gpurun_out/r6ap/bench.err || { tail -30 gpurun_out/r6ap/bench.err; exit 1; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r6ap/bench.json"))
c1 = d["configs"]["C1_EC6P6_1MiB_encode"]
print({k: v for k, v in c1.items() if k not in ("workload", "gate")}, d["value"], d.get("gate_failures"))
PY
exit 0
