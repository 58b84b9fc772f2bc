# Build a variant of libcfsec.so with extra -D flags for the fused CRC kernels (A/B probes):
#   bash tools/build_variant.sh <name> <flags...>   ->  probes_bin/<name>/libcfsec.so + gf_shapes
# Reuses build/cfsec/*.o (make first) except the units in $UNITS (default: the CRC kernels).
set -e
name=$1; shift
out=probes_bin/$name; mkdir -p $out/obj
HIPCC=/opt/rocm/bin/hipcc
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result $*"
objs=""
UNITS=${UNITS:-"gf_crc gf_crc_k6 gf_crc_k8 gf_crc_k12 gf_crc_k16 gf_crc_k18 crc32 crc32block"}
for k in $UNITS; do
  $HIPCC $F -c chubaofs_amd/csrc/$k.hip -o $out/obj/$k.o &
  objs="$objs $out/obj/$k.o"
done
wait
for o in build/cfsec/*.o; do case " $UNITS " in *" $(basename $o .o) "*) ;; *) objs="$objs $o";; esac; done
$HIPCC --offload-arch=gfx950 -shared -fPIC -o $out/libcfsec.so $objs
$HIPCC --offload-arch=gfx950 -O3 -std=c++17 -Ichubaofs_amd/csrc tools/gf_shapes.hip -L$out -lcfsec -Wl,-rpath,'$ORIGIN' -o $out/gf_shapes
rm -rf $out/obj
