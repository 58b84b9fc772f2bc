# Round 6, session Y: the C5 repair's in-pass checksum form (CFSEC_BS_REPAIR_CRC=1) in per-stripe tile
# order (W waves per bid, every W-th tile; the Horner jump rebuilt for 2048 W bytes) instead of blocks:
# its tests, then C5's tasklet with the separate pass (default) and with the in-pass form.
set -o pipefail
mkdir -p gpurun_out/r6y
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bs_crc.py \
  tests/test_gpu_batch.py -k "crc or repair or reconstruct" > gpurun_out/r6y/pytest.log 2>&1 || { tail -40 gpurun_out/r6y/pytest.log; exit 1; }
tail -1 gpurun_out/r6y/pytest.log
for v in 0 1 0 1; do
  echo "== CFSEC_BS_REPAIR_CRC=$v" >> gpurun_out/r6y/c5.txt
  CFSEC_BS_REPAIR_CRC=$v timeout -k 10 120 python tools/c5_crc_probe.py >> gpurun_out/r6y/c5.txt 2>&1 || exit $?
done
grep -E "==|us per call|all" gpurun_out/r6y/c5.txt
exit 0
