# Round-3 evidence for DESIGN §7: the two PMC passes of tools/pmc_ab.sh (one counter group per run)
# over C5's tasklet (tools/c5_crc_probe.py: gf_dy16_repair_kernel<2, 2> + the CRC pass) and the
# shape sweep (the fused encode + CRC lookup kernel, the EC16P20(L2) dyadic kernels).
set -e
export TMPDIR=/tmp GF_SHAPES_REPS=3 GF_SHAPES_NOSETTLE=1 C5_REPS=5
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
mkdir -p gpurun_out
timeout -s KILL 150 rocprofv3 --pmc $P1 -d gpurun_out/pmc_c5_1 -o run --output-format csv -- python3 tools/c5_crc_probe.py > gpurun_out/pmc_c5_1.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc $P2 -d gpurun_out/pmc_c5_2 -o run --output-format csv -- python3 tools/c5_crc_probe.py > gpurun_out/pmc_c5_2.log 2>&1
python3 tools/pmc_summary.py gpurun_out/pmc_c5_1 > gpurun_out/pmc_c5.txt
python3 tools/pmc_summary.py gpurun_out/pmc_c5_2 >> gpurun_out/pmc_c5.txt
timeout -s KILL 150 rocprofv3 --pmc $P1 -d gpurun_out/pmc_sh_1 -o run --output-format csv -- tools/gf_shapes > gpurun_out/pmc_sh_1.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc $P2 -d gpurun_out/pmc_sh_2 -o run --output-format csv -- tools/gf_shapes > gpurun_out/pmc_sh_2.log 2>&1
python3 tools/pmc_summary.py gpurun_out/pmc_sh_1 > gpurun_out/pmc_shapes.txt
python3 tools/pmc_summary.py gpurun_out/pmc_sh_2 >> gpurun_out/pmc_shapes.txt
