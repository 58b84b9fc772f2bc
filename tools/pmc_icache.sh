# Instruction-fetch counters per kernel over gf_shapes (one pass per counter group; SQC one counter
# per pass).  Output: gpurun_out/pmc_ic_<pass>/ and gpurun_out/pmc_ic.txt.
set -e
export TMPDIR=/tmp GF_SHAPES_REPS=3 GF_SHAPES_NOSETTLE=1
B=./probes_bin/gf_shapes_main
timeout -s KILL 90 rocprofv3 --pmc SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_BUSY_CYCLES -d gpurun_out/pmc_ic_a -o run --output-format csv -- $B > gpurun_out/pmc_ic_a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_MISSES -d gpurun_out/pmc_ic_b -o run --output-format csv -- $B > gpurun_out/pmc_ic_b.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS -d gpurun_out/pmc_ic_c -o run --output-format csv -- $B > gpurun_out/pmc_ic_c.log 2>&1
for p in a b c; do python3 tools/pmc_summary.py gpurun_out/pmc_ic_$p; done > gpurun_out/pmc_ic.txt
