# Variants of the bit-sliced repair kernel (tools/build_variant.sh builds): C5's tasklet per call
# with and without checksums, and the repair kernel's trace median, one library at a time.
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/r4_bs_rep_var.txt
: > $out
cp chubaofs_amd/libcfsec.so gpurun_out/lib_default.so
for v in default bs_old default bs_old; do
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
done
cp gpurun_out/lib_default.so chubaofs_amd/libcfsec.so
rm -f gpurun_out/lib_default.so
rm -rf gpurun_out/var_*
cat $out
