# Round 6, session AH: the host cost of an asynchronous batch call before / after the workspace
# acquire stops querying every pending workspace's event (tools/libcfsec_oldacq.so: the old acquire).
set -o pipefail
mkdir -p gpurun_out/r6ah
export TMPDIR=/tmp
for lib in tools/libcfsec_oldacq.so chubaofs_amd/libcfsec.so tools/libcfsec_oldacq.so chubaofs_amd/libcfsec.so; do
  echo "== $lib" >> gpurun_out/r6ah/host.txt
  CFSEC_LIB_PATH=$PWD/$lib timeout -k 10 120 python tools/host_call_cost.py EC6P10L2 >> gpurun_out/r6ah/host.txt 2>&1 || { cat gpurun_out/r6ah/host.txt; exit 1; }
  CFSEC_LIB_PATH=$PWD/$lib timeout -k 10 120 python tools/host_call_cost.py EC12P4 5592406 8 >> gpurun_out/r6ah/host.txt 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/r6ah/host.txt
exit 0
