# Round 6, session AY (closing, final library incl. the crc32block grid): the full GPU suite + smoke on the shipped library (every code mode's encode
# + checksums fused), the C-ABI latency tool, the driver's bench line, a kernel-trace profile of the
# same bench with the timed-region statistics, the shape sweep, and the N = 2 rehearsal (gloo, the
# box's one GPU shared by both ranks).
set -o pipefail
mkdir -p gpurun_out/r6j
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ \
  > gpurun_out/r6j/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/r6j/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r6j/pytest_gpu.log
timeout -k 10 120 python -c 'import __graft_entry__ as g; g.smoke()' 2>&1 | tail -1
timeout -k 10 120 ./tools/seg_latency 200 null > gpurun_out/r6j/seg_latency_null.json 2>&1 || exit $?
timeout -k 10 500 python bench.py > gpurun_out/r6j/bench.json 2> gpurun_out/r6j/bench.err; rc=$?
echo "bench rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 3 ] || { tail -20 gpurun_out/r6j/bench.err; exit $rc; }
timeout -k 10 450 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6j/prof -o run -- python3 bench.py --no-cpu --no-pmc > gpurun_out/r6j/bench_prof.json 2> gpurun_out/r6j/bench_prof.err; rc=$?
echo "prof rc=$rc"; [ $rc -eq 0 ] || [ $rc -eq 3 ] || exit $rc
python tools/timed_region_stats.py gpurun_out/r6j/prof gpurun_out/r6j/bench_prof.json gpurun_out/r6j/timed_region_stats.txt
head -6 gpurun_out/r6j/timed_region_stats.txt
timeout -k 10 200 ./tools/gf_shapes > gpurun_out/r6j/shape_sweep.txt 2>&1 || exit $?
CFSEC_BENCH_SHARE_DEVICE=1 CFSEC_BENCH_BACKEND=gloo timeout -k 10 500 python bench.py --gpus 2 --no-cpu --no-pmc \
  > gpurun_out/r6j/bench_n2_shared_gpu_rehearsal.json 2> gpurun_out/r6j/bench_n2.err; rc=$?
echo "n2 rc=$rc"
python3 - <<'PY'
import json
d = json.load(open("gpurun_out/r6j/bench.json"))
c4 = d["configs"]["C4_EC6P10L2_lrc_encode_local_repair"]; c5 = d["configs"]["C5_EC16P20L2_repair_tasklet"]
print("value", d["value"], "frac", d["roofline"]["frac"], "traffic", d["roofline"]["traffic"], "enc_crc", d.get("encode_crc_roofline_frac"),
      "seam", d.get("ec_seam_encode_crc_roofline_frac"), "C4 crc", c4.get("encode_crc_kernel_roofline_frac"),
      "C5", c5.get("kernel_roofline_frac"), c5.get("with_crc_over_kernel"), "gate", d.get("gate_failures"))
try:
    n2 = json.load(open("gpurun_out/r6j/bench_n2_shared_gpu_rehearsal.json"))
    print("n2", n2["value"], n2.get("gate_failures"))
except Exception as e:
    print("n2 parse", e)
PY
exit 0
