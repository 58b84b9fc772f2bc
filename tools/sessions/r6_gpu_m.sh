# Round 6, session M: what bounds the per-row form of C4's fused encode + 18 checksums -- 4 waves per
# SIMD (spills), the next tile's inputs loaded before the network (2 waves), and timing probes without
# any checksum lookups (CFSEC_BC_PROBE=3: wrong words, timing only).
set -o pipefail
mkdir -p gpurun_out/r6m
export TMPDIR=/tmp
for v in base pr_w4 pr_pf2 pr_probe3 pr_probe3_pf2; do
  lib=chubaofs_amd/libcfsec.so; [ $v = base ] || lib=probes_bin/$v/libcfsec.so
  echo "== $v" >> gpurun_out/r6m/c4.txt
  CFSEC_LIB_PATH=$PWD/$lib CFSEC_BS_CRC=5 timeout -k 10 120 python tools/c4_crc_probe.py >> gpurun_out/r6m/c4.txt 2>&1
  rc=$?; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
grep -E "==|us per call|all" gpurun_out/r6m/c4.txt
# PMC over the per-row form (tools/r5_pmc_crc.sh's counter groups), one group per run
export C4_REPS=5
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for p in 1 2; do
  eval P=\$P$p
  CFSEC_BS_CRC=5 timeout -s KILL 150 rocprofv3 --pmc $P -d gpurun_out/r6m/pmc_$p -o run --output-format csv -- python3 tools/c4_crc_probe.py > gpurun_out/r6m/pmc_$p.log 2>&1 || exit $?
done
python3 tools/pmc_summary.py gpurun_out/r6m/pmc_1 > gpurun_out/r6m/pmc_c4_bs.txt
python3 tools/pmc_summary.py gpurun_out/r6m/pmc_2 >> gpurun_out/r6m/pmc_c4_bs.txt
cat gpurun_out/r6m/pmc_c4_bs.txt
exit 0
