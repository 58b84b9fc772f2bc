# round-5 session J: C4's local repair (k = 8, m = 1 store) with 2 / 4 / 8 rows of lookahead
set -o pipefail
mkdir -p gpurun_out/r5
for i in 1 2; do
  timeout -k 10 120 python3 tools/c4_local_probe.py > gpurun_out/r5/c4l_d2_$i.txt 2>&1 && \
  CFSEC_LIB_PATH=probes_bin/r5_fixd4/libcfsec.so timeout -k 10 120 python3 tools/c4_local_probe.py > gpurun_out/r5/c4l_d4_$i.txt 2>&1 && \
  CFSEC_LIB_PATH=probes_bin/r5_fixd8/libcfsec.so timeout -k 10 120 python3 tools/c4_local_probe.py > gpurun_out/r5/c4l_d8_$i.txt 2>&1 || exit $?
done
for f in gpurun_out/r5/c4l_*.txt; do echo "$f: $(grep sync $f)"; done
