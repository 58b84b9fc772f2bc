# round-5 session T: which kernels test_reconstruct_stripes_mock_bids[10-4-device] runs
set -o pipefail
mkdir -p gpurun_out/r5
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5/mockprof -o mock -- python3 -m pytest -q -m gpu "tests/test_gpu_batch.py::test_reconstruct_stripes_mock_bids[10-4-device]" > gpurun_out/r5/mockprof.log 2>&1
cut -d, -f1-2 gpurun_out/r5/mockprof/mock_kernel_stats.csv | grep -v 'at::' | cut -c1-160
