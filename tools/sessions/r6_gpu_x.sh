# Round 6, session X: the C5 repair kernel's tiles in per-stripe order (W waves per bid, every W-th
# tile: the order a per-row checksum run needs) against its every-nw-th-tile order; C5's tasklet.
set -o pipefail
mkdir -p gpurun_out/r6x
export TMPDIR=/tmp
for v in base perbid base perbid; do
  lib=chubaofs_amd/libcfsec.so; [ $v = base ] || lib=probes_bin/$v/libcfsec.so
  echo "== $v" >> gpurun_out/r6x/c5.txt
  CFSEC_LIB_PATH=$PWD/$lib timeout -k 10 120 python tools/c5_crc_probe.py >> gpurun_out/r6x/c5.txt 2>&1 || exit $?
done
grep -E "==|us per call|all" gpurun_out/r6x/c5.txt
exit 0
