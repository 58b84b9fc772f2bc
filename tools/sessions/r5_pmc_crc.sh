# Round-5 PMC passes over the fused encode + checksum kernels VERDICT r4 names (What's weak #2, #3):
# C4's gf_crc_kernel<6,12,true,2,2> beside the plain gf_dy_kernel<6,12,...> (tools/c4_crc_probe.py),
# and EC12P4's gf_crc_lds_kernel<12,4,true> beside its plain encode (tools/ec_crc_probe.py).
# One counter group per run (rocprofv3 does not split passes).
set -o pipefail
export TMPDIR=/tmp C4_REPS=5 EC_REPS=5
mkdir -p gpurun_out/r5
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for probe in c4_crc_probe ec_crc_probe; do
  for p in 1 2; do
    eval P=\$P$p
    timeout -s KILL 150 rocprofv3 --pmc $P -d gpurun_out/r5/pmc_${probe}_$p -o run --output-format csv -- python3 tools/$probe.py > gpurun_out/r5/pmc_${probe}_$p.log 2>&1 || exit $?
  done
  python3 tools/pmc_summary.py gpurun_out/r5/pmc_${probe}_1 > gpurun_out/r5/pmc_$probe.txt
  python3 tools/pmc_summary.py gpurun_out/r5/pmc_${probe}_2 >> gpurun_out/r5/pmc_$probe.txt
done
timeout -k 10 120 python3 tools/c4_crc_probe.py > gpurun_out/r5/c4_crc_probe.txt 2>&1
cat gpurun_out/r5/pmc_c4_crc_probe.txt gpurun_out/r5/c4_crc_probe.txt
