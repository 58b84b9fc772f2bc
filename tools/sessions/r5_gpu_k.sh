# round-5 session K: C4's local repair (k = 8, m = 1 store), 1 / 2 / 4 / 8 tiles per workgroup
set -o pipefail
mkdir -p gpurun_out/r5
for i in 1 2; do
  timeout -k 10 120 python3 tools/c4_local_probe.py > gpurun_out/r5/c4t_1_$i.txt 2>&1 || exit $?
  for t in 2 4 8; do
    CFSEC_LIB_PATH=probes_bin/r5_tpw$t/libcfsec.so timeout -k 10 120 python3 tools/c4_local_probe.py > gpurun_out/r5/c4t_${t}_$i.txt 2>&1 || exit $?
  done
done
for f in gpurun_out/r5/c4t_*.txt; do echo "$f: $(grep -E 'sync|async' $f | tr '\n' ' ')"; done
# the checksum pass over C5's rebuilt rows: shipped form vs AHEAD 4 / 16 and the two timing-only cuts
for v in base a4 a16 d1 d2; do
  b=tools/crc_pass_probe; [ $v = base ] || b=probes_bin/r5_crc_$v/crc_pass_probe
  echo "== $v" >> gpurun_out/r5/crc_pass_k.txt
  timeout -k 10 120 $b >> gpurun_out/r5/crc_pass_k.txt 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r5/crcprof -o crc -- tools/crc_pass_probe > gpurun_out/r5/crcprof.log 2>&1 || exit $?
cat gpurun_out/r5/crc_pass_k.txt
