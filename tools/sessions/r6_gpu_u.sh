# Round 6, session U: every route of the bit-sliced fused encode + checksums on by default (EC12P4 for
# rows of >= 2 MiB): the full GPU suite and smoke, then the bench (its encode + CRC fields now on the
# bit-sliced kernel for EC12P4's 64 MiB blobs and C4).
set -o pipefail
mkdir -p gpurun_out/r6u
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r6u/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r6u/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r6u/pytest_gpu.log
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' 2>&1 | tail -1
timeout -k 10 500 python bench.py > gpurun_out/r6u/bench.json 2> gpurun_out/r6u/bench.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 3 ] || { tail -20 gpurun_out/r6u/bench.err; exit $rc; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r6u/bench.json"))
print(d["value"], d["roofline"]["frac"], "enc_crc", d.get("encode_crc_roofline_frac"), "seam", d.get("ec_seam_encode_crc_roofline_frac"))
c4 = d["configs"]["C4_EC6P10L2_lrc_encode_local_repair"]
print("C4 encode_crc", c4.get("encode_crc_kernel_ms"), c4.get("encode_crc_kernel_roofline_frac"))
c5 = d["configs"]["C5_EC16P20L2_repair_tasklet"]
print("C5", c5.get("kernel_roofline_frac"), c5.get("with_crc_over_kernel"), "gate_failures", d.get("gate_failures"))
PY
exit 0
