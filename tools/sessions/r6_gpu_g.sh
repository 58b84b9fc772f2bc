# Round 6, session G: where the second-phase checksum form's time goes -- C5's call with phase 2
# (shipped form), with its atomics replaced by plain stores (r6_p2a, wrong words), and with phase 2
# compiled out of the P2 kernel (r6_p2b), against the separate pass; alternated twice.
set -o pipefail
mkdir -p gpurun_out/r6g
for i in 1 2; do
  timeout -k 10 120 python3 tools/c5_crc_probe.py > gpurun_out/r6g/c5_sep_$i.txt 2>&1 && \
  CFSEC_BS_REPAIR_CRC=2 timeout -k 10 120 python3 tools/c5_crc_probe.py > gpurun_out/r6g/c5_p2_$i.txt 2>&1 && \
  C5_NOCHECK=1 CFSEC_BS_REPAIR_CRC=2 CFSEC_LIB_PATH=$PWD/probes_bin/r6_p2a/libcfsec.so timeout -k 10 120 python3 tools/c5_crc_probe.py > gpurun_out/r6g/c5_p2a_$i.txt 2>&1 && \
  C5_NOCHECK=1 CFSEC_BS_REPAIR_CRC=2 CFSEC_LIB_PATH=$PWD/probes_bin/r6_p2b/libcfsec.so timeout -k 10 120 python3 tools/c5_crc_probe.py > gpurun_out/r6g/c5_p2b_$i.txt 2>&1 || exit $?
done
for f in gpurun_out/r6g/c5_*.txt; do echo "== $f"; grep "us per call\|bids" $f | tr '\n' ' '; echo; done
