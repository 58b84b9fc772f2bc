# Round 6, session H: the second-phase checksum form with the tile-to-row-end multiply per lane from
# scalar columns (no bit-serial scalar multiply): its GPU tests, then C5's call against the separate pass.
set -o pipefail
mkdir -p gpurun_out/r6h
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bs_crc.py \
  > gpurun_out/r6h/pytest_bs_crc.log 2>&1 || { tail -40 gpurun_out/r6h/pytest_bs_crc.log; exit 1; }
tail -1 gpurun_out/r6h/pytest_bs_crc.log
for i in 1 2; do
  timeout -k 10 120 python3 tools/c5_crc_probe.py > gpurun_out/r6h/c5_sep_$i.txt 2>&1 && \
  CFSEC_BS_REPAIR_CRC=2 timeout -k 10 120 python3 tools/c5_crc_probe.py > gpurun_out/r6h/c5_p2_$i.txt 2>&1 || exit $?
done
for f in gpurun_out/r6h/c5_*.txt; do echo "== $f"; grep "us per call\|bids" $f | tr '\n' ' '; echo; done
