# round-5 session H: the 4-op swapmove (gf_bitslice.hpp CFSEC_BS_SWAP) A/B: bit-sliced GPU tests,
# the shape sweep (EC16P20 / EC16P20L2 encode, Verify) and C5's repair tasklet, alternated twice
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_batch.py tests/test_gpu_bs_crc.py tests/test_gpu_parity.py -k "16 or bs or scattered or tasklet" > gpurun_out/r5/test_swap.log 2>&1; rc=$?
tail -3 gpurun_out/r5/test_swap.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 ./tools/gf_shapes > gpurun_out/r5/shapes_swap1_$i.txt 2>&1 && \
  timeout -k 10 200 ./probes_bin/r5_swap0/gf_shapes > gpurun_out/r5/shapes_swap0_$i.txt 2>&1 && \
  timeout -k 10 120 python3 tools/c5_crc_probe.py > gpurun_out/r5/c5_swap1_$i.txt 2>&1 && \
  CFSEC_LIB_PATH=probes_bin/r5_swap0/libcfsec.so timeout -k 10 120 python3 tools/c5_crc_probe.py > gpurun_out/r5/c5_swap0_$i.txt 2>&1 || exit $?
done
for f in gpurun_out/r5/shapes_swap*_*.txt; do echo "== $f"; grep -i 'EC16P20' $f; done
for f in gpurun_out/r5/c5_swap*_*.txt; do echo "== $f"; grep 'per call' $f | tail -2; done
