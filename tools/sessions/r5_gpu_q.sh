# round-5 session Q: the table-launch repair kernel on C5's contiguous layout (CFSEC_BS_FORCE_TAB=1):
# is the scattered call's slower kernel the table or the layout?
set -o pipefail
mkdir -p gpurun_out/r5
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
out=gpurun_out/r5/force_tab.txt
echo "== default" > $out
C5_REPS=30 timeout -k 10 120 python3 tools/c5_scatter_probe.py >> $out 2>&1 || exit $?
echo "== CFSEC_BS_FORCE_TAB=1" >> $out
CFSEC_BS_FORCE_TAB=1 C5_REPS=30 timeout -k 10 120 python3 tools/c5_scatter_probe.py >> $out 2>&1 || exit $?
CFSEC_BS_FORCE_TAB=1 C5_REPS=30 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/force_tab -o ft -- python3 tools/c5_scatter_probe.py > gpurun_out/r5/force_tab.log 2>&1 || exit $?
grep repair_kernel gpurun_out/r5/force_tab/ft_kernel_stats.csv | cut -c1-250 >> $out
cat $out
echo "== CFSEC_BS_VOFF=1 (probes_bin/r5_voff)" >> $out
CFSEC_LIB_PATH=probes_bin/r5_voff/libcfsec.so C5_REPS=30 timeout -k 10 120 python3 tools/c5_scatter_probe.py >> $out 2>&1 || exit $?
CFSEC_LIB_PATH=probes_bin/r5_voff/libcfsec.so C5_REPS=30 timeout -k 10 120 python3 tools/c5_scatter_probe.py >> $out 2>&1 || exit $?
cat $out
