# Round 6, session I: the standalone checksum pass with the alignment basis requested before the tiles
# (short runs: C5's 256 rebuilt rows) against the late load (r6_crclate): C5's call with checksums and
# the sweep's crc-only column, alternated; the CRC GPU tests on the current library.
set -o pipefail
mkdir -p gpurun_out/r6i
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_crc.py \
  tests/test_gpu_bs_crc.py > gpurun_out/r6i/pytest_crc.log 2>&1 || { tail -40 gpurun_out/r6i/pytest_crc.log; exit 1; }
tail -1 gpurun_out/r6i/pytest_crc.log
for i in 1 2; do
  timeout -k 10 120 python3 tools/c5_crc_probe.py > gpurun_out/r6i/c5_early_$i.txt 2>&1 && \
  CFSEC_LIB_PATH=$PWD/probes_bin/r6_crclate/libcfsec.so timeout -k 10 120 python3 tools/c5_crc_probe.py > gpurun_out/r6i/c5_late_$i.txt 2>&1 || exit $?
done
timeout -k 10 200 ./tools/gf_shapes > gpurun_out/r6i/shapes_early.txt 2>&1 && \
timeout -k 10 200 ./probes_bin/r6_crclate/gf_shapes > gpurun_out/r6i/shapes_late.txt 2>&1 || exit $?
for f in gpurun_out/r6i/c5_*.txt; do echo "== $f"; grep "us per call" $f | tail -2 | tr '\n' ' '; echo; done
paste <(awk '{print $1, $2, $NF-0, $(NF-1)}' gpurun_out/r6i/shapes_early.txt) <(awk '{print $(NF-1)}' gpurun_out/r6i/shapes_late.txt) | head -25
