# A/B of bit-sliced kernel variants (libraries from tools/build_variant.sh under probes_bin/<name>;
# "default" = the in-tree library): C5's tasklet per call, its repair kernel's trace median and the
# shape sweep's EC16P20 / EC16P20L2 rows, libraries alternated twice.
#   bash tools/r4_bs_var_ab.sh <out name> <variant>...
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/$1.txt; shift
: > $out
cp chubaofs_amd/libcfsec.so gpurun_out/lib_default.so
for v in "$@" "$@"; do
  if [ $v = default ]; then cp gpurun_out/lib_default.so chubaofs_amd/libcfsec.so; else cp probes_bin/$v/libcfsec.so chubaofs_amd/libcfsec.so; fi
  echo "== $v" >> $out
  timeout -k 10 200 python tools/c5_crc_probe.py 2>/dev/null | grep -v amdgpu >> $out
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/var_$v -o run -- python3 tools/c5_crc_probe.py > /dev/null 2>&1
  python3 - "$v" >> $out <<'PY'
import csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(f"gpurun_out/var_{sys.argv[1]}/run_kernel_trace.csv")[0])))
for key in ("bs16_repair", "crc32_horner"):
    d = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows if key in r["Kernel_Name"])
    if d:
        print(f"  {key}: n={len(d)} median {d[len(d)//2]:.1f} us  p10 {d[len(d)//10]:.1f}  p90 {d[9*len(d)//10]:.1f}")
PY
  rm -rf gpurun_out/var_$v
  timeout -k 10 150 tools/gf_shapes | grep -E "EC16P20 global|EC16P20L2 fused" >> $out
done
cp gpurun_out/lib_default.so chubaofs_amd/libcfsec.so
rm -f gpurun_out/lib_default.so
cat $out
