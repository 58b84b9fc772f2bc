# Round 6, session AJ (after the tail waves): the bench's EC12P4 encode + checksum legs (fused encode_crc_batch and the ec seam)
# with EC12P4's bit-sliced route off (CFSEC_BS_CRC=53, the default) and on (55), twice each, same box.
set -o pipefail
mkdir -p gpurun_out/r6aj
export TMPDIR=/tmp
for v in 53 55 53 55; do
  CFSEC_BS_CRC=$v timeout -k 10 300 python bench.py --no-cpu --no-pmc > gpurun_out/r6aj/bench_$v.json 2> gpurun_out/r6aj/bench_$v.err || exit $?
  python3 - "$v" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/r6aj/bench_{sys.argv[1]}.json"))
c4 = d["configs"]["C4_EC6P10L2_lrc_encode_local_repair"]
print("mask", sys.argv[1], "enc_crc", d.get("encode_crc_roofline_frac"), "seam", d.get("ec_seam_encode_crc_roofline_frac"),
      "seam_ms", d.get("ec_seam_encode_crc_ms"), "C4", c4.get("encode_crc_kernel_roofline_frac"), "value", d["value"])
PY
done
exit 0
