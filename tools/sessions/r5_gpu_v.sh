# round-5 session V: PMC of the library's fixed-K (8, 1) kernel vs the probe's register-table kernel
set -o pipefail
mkdir -p gpurun_out/r5
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES --output-format csv -d gpurun_out/r5/pmc_c4l -o p1 -- tools/c4l_pattern_probe > gpurun_out/r5/pmc_c4l1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TA_BUSY_avr TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d gpurun_out/r5/pmc_c4l -o p2 -- tools/c4l_pattern_probe > gpurun_out/r5/pmc_c4l2.log 2>&1 || exit $?
ls gpurun_out/r5/pmc_c4l
