# Round 6: the full GPU suite + smoke with every bit-sliced route at its default (CFSEC_BS_CRC=53),
# then the bench line once more.
set -o pipefail
mkdir -p gpurun_out/r6ab
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r6ab/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r6ab/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r6ab/pytest_gpu.log
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' 2>&1 | tail -1
timeout -k 10 500 python bench.py > gpurun_out/r6ab/bench.json 2> gpurun_out/r6ab/bench.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 3 ] || { tail -20 gpurun_out/r6ab/bench.err; exit $rc; }
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r6ab/bench.json"))
c4 = d["configs"]["C4_EC6P10L2_lrc_encode_local_repair"]; c5 = d["configs"]["C5_EC16P20L2_repair_tasklet"]
print("value", d["value"], "frac", d["roofline"]["frac"], "enc_crc", d.get("encode_crc_roofline_frac"),
      "seam", d.get("ec_seam_encode_crc_roofline_frac"), "C4 crc", c4.get("encode_crc_kernel_roofline_frac"),
      "C5", c5.get("kernel_roofline_frac"), c5.get("with_crc_over_kernel"), "gate", d.get("gate_failures"))
PY
exit 0
