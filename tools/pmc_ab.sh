# PMC passes (one counter group per run) over two probe binaries: $1 and $2 (paths), output under
# gpurun_out/pmc_<name>_<pass>/.  GF_SHAPES_REPS keeps the dispatch count small.
set -e
export TMPDIR=/tmp GF_SHAPES_REPS=${GF_SHAPES_REPS:-3} GF_SHAPES_NOSETTLE=1
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for b in "$@"; do
  n=$(basename $b)
  timeout -s KILL 120 rocprofv3 --pmc $P1 -d gpurun_out/pmc_${n}_1 -o run --output-format csv -- $b > gpurun_out/pmc_${n}_1.log 2>&1
  timeout -s KILL 120 rocprofv3 --pmc $P2 -d gpurun_out/pmc_${n}_2 -o run --output-format csv -- $b > gpurun_out/pmc_${n}_2.log 2>&1
  python3 tools/pmc_summary.py gpurun_out/pmc_${n}_1 > gpurun_out/pmc_${n}.txt
  python3 tools/pmc_summary.py gpurun_out/pmc_${n}_2 >> gpurun_out/pmc_${n}.txt
done
