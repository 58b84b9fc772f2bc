# Round 6, session F: the second-phase checksum form of the bit-sliced repair (CFSEC_BS_REPAIR_CRC=2):
# its GPU tests (both repair-pass forms, every layout), then C5's tasklet with the separate pass, the
# round-5 in-network form and the second phase, alternated, every bid's words checked against zlib.
set -o pipefail
mkdir -p gpurun_out/r6f
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_bs_crc.py \
  tests/test_gpu_batch.py -k "crc or 16_20 or scattered" > gpurun_out/r6f/pytest_bs_crc.log 2>&1 \
  || { tail -40 gpurun_out/r6f/pytest_bs_crc.log; exit 1; }
tail -1 gpurun_out/r6f/pytest_bs_crc.log
for i in 1 2; do
  timeout -k 10 120 python3 tools/c5_crc_probe.py > gpurun_out/r6f/c5_sep_$i.txt 2>&1 && \
  CFSEC_BS_REPAIR_CRC=2 timeout -k 10 120 python3 tools/c5_crc_probe.py > gpurun_out/r6f/c5_p2_$i.txt 2>&1 && \
  CFSEC_BS_REPAIR_CRC=1 timeout -k 10 120 python3 tools/c5_crc_probe.py > gpurun_out/r6f/c5_inline_$i.txt 2>&1 || exit $?
done
for f in gpurun_out/r6f/c5_*.txt; do echo "== $f"; grep "us per call\|bids" $f | tr '\n' ' '; echo; done
