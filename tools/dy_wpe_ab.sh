# Round-3 probe: waves-per-EU floor of the k = 12 dyadic kernels (98 VGPRs / 4 waves shipped vs 96 / 5
# waves with 3 spilled VGPRs): the bench headline in the rotated batches, alternated, same box.
set -e
mkdir -p gpurun_out
for v in base wpe5 base wpe5; do
  lib=chubaofs_amd/libcfsec.so; [ $v = base ] || lib=probes_bin/$v/libcfsec.so
  echo "== $v" >> gpurun_out/dy_wpe_ab.txt
  CFSEC_LIB_PATH=$lib timeout -k 10 240 python bench.py --no-cpu --no-pmc --no-extra --steps 40 > gpurun_out/dy_wpe_$v.json
  python -c "import json,sys;b=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(b['value'],b['ms_per_step'],b['roofline']['frac'])" gpurun_out/dy_wpe_$v.json >> gpurun_out/dy_wpe_ab.txt
done
