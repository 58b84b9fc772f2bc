# round-5 session P: where the scattered C5 call's 11 us gap + 4.7 us copy go (table upload A/B)
set -o pipefail
mkdir -p gpurun_out/r5
out=gpurun_out/r5/scat_upload_ab.txt
timeout -k 10 60 tools/fg_probe > $out 2>&1 || exit $?
for v in base diag1 diag2 host; do
  echo "== $v" >> $out
  case $v in
    base) C5_REPS=50 timeout -k 10 120 python3 tools/c5_scatter_probe.py >> $out 2>&1 || exit $? ;;
    diag1) CFSEC_BS_DTAB_DIAG=1 C5_REPS=50 timeout -k 10 120 python3 tools/c5_scatter_probe.py >> $out 2>&1 || exit $? ;;
    diag2) CFSEC_BS_DTAB_DIAG=2 C5_REPS=50 timeout -k 10 120 python3 tools/c5_scatter_probe.py >> $out 2>&1 || exit $? ;;
    host) CFSEC_BS_DTAB_HOST=1 C5_REPS=50 timeout -k 10 120 python3 tools/c5_scatter_probe.py >> $out 2>&1 || exit $? ;;
  esac
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
CFSEC_BS_DTAB_DIAG=2 C5_REPS=30 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r5/scat_trace2 -o scat -- python3 tools/c5_scatter_probe.py > gpurun_out/r5/scat_trace2.log 2>&1 || exit $?
n=$(python3 tools/trace_timeline.py gpurun_out/r5/scat_trace2 --count 100000 | wc -l)
python3 tools/trace_timeline.py gpurun_out/r5/scat_trace2 --skip $((n - 60)) --count 20 >> $out
cat $out
