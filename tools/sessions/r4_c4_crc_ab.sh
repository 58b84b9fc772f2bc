# Round 4: C4's encode + 18 checksums, fused kernel (default) vs the separate pass
set -e
mkdir -p gpurun_out
for rep in 1 2; do
  echo "fused" >> gpurun_out/r4_c4_crc_ab.txt
  timeout -k 10 120 python3 tools/c4_crc_probe.py >> gpurun_out/r4_c4_crc_ab.txt 2>&1
  echo "separate pass (CFSEC_BATCH_FUSED_CRC=0)" >> gpurun_out/r4_c4_crc_ab.txt
  CFSEC_BATCH_FUSED_CRC=0 timeout -k 10 120 python3 tools/c4_crc_probe.py >> gpurun_out/r4_c4_crc_ab.txt 2>&1
done
for rep in 1 2; do
  echo "fused, byte-table step (probes_bin/step0)" >> gpurun_out/r4_c4_crc_ab2.txt
  CFSEC_LIB_PATH=probes_bin/step0/libcfsec.so timeout -k 10 120 python3 tools/c4_crc_probe.py >> gpurun_out/r4_c4_crc_ab2.txt 2>&1
  echo "fused, 5-bit step (default)" >> gpurun_out/r4_c4_crc_ab2.txt
  timeout -k 10 120 python3 tools/c4_crc_probe.py >> gpurun_out/r4_c4_crc_ab2.txt 2>&1
done
