# Round-5 stale-DMA reproduction (tools/r5_stale_dma_probe.py): the round-4 kernels (no exit drain)
# and the fixed ones, two streams of one process and two processes sharing the GPU.
set -o pipefail
mkdir -p gpurun_out/r5
P=tools/r5_stale_dma_probe.py
ND=probes_bin/r5_nodrain_dbg/libcfsec.so
DR=probes_bin/r5_drain_dbg/libcfsec.so
run() { # name lib args...
  local name=$1 lib=$2; shift 2
  timeout -k 10 240 env CFSEC_LIB_PATH=$lib python -u $P "$@" > gpurun_out/r5/probe_$name.json 2> gpurun_out/r5/probe_$name.err
}
run nodrain_s2 $ND --streams 2 --iters 6000 && \
run nodrain_p2 $ND --streams 1 --procs 2 --iters 6000 && \
run drain_s2 $DR --streams 2 --iters 6000 && \
run drain_p2 $DR --streams 1 --procs 2 --iters 6000
rc=$?
for f in gpurun_out/r5/probe_*_[sp]2.json; do echo "$f"; python -c "import json,sys; d=json.load(open('$f')); print(d['false_verify_calls'])"; done
exit $rc
