# Round-4 evidence: the two PMC passes of tools/pmc_c5.sh (one counter group per run) over C5's
# tasklet (tools/c5_crc_probe.py) with the final library: the bit-sliced repair kernel
# (gf_bs16_repair_kernel<22, 2>) and the checksum pass.
set -e
export TMPDIR=/tmp C5_REPS=5
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
mkdir -p gpurun_out
timeout -s KILL 150 rocprofv3 --pmc $P1 -d gpurun_out/pmc_bs_1 -o run --output-format csv -- python3 tools/c5_crc_probe.py > gpurun_out/pmc_bs_1.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc $P2 -d gpurun_out/pmc_bs_2 -o run --output-format csv -- python3 tools/c5_crc_probe.py > gpurun_out/pmc_bs_2.log 2>&1
python3 tools/pmc_summary.py gpurun_out/pmc_bs_1 > gpurun_out/pmc_c5_bs.txt
python3 tools/pmc_summary.py gpurun_out/pmc_bs_2 >> gpurun_out/pmc_c5_bs.txt
