#!/bin/bash
# Re-link an A/B variant library after host-side (slm_capi.hip) changes: recompile
# its slm_capi.o with the variant's flags, keep its kernel objects.
# usage: tools/relink_variant.sh <name> "<EXTRA flags>" <plan keys...>
set -e
name=$1; extra=$2; shift 2
root=$(cd $(dirname $0)/.. && pwd)
src=$root/spatial_light_modulator_module_amd/csrc
base=$root/build/csrc
out=$root/build/var_$name
objs=""
for f in $base/kernels_*.o; do
  k=$(basename $f .o); k=${k#kernels_}
  if [[ " $* " == *" $k "* ]]; then objs="$objs $out/kernels_$k.o"; else objs="$objs $f"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=fast -fno-slp-vectorize -Wno-unused-function $extra -I/opt/rocm/include -c $src/slm_capi.hip -o $out/slm_capi.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $root/spatial_light_modulator_module_amd/lib/libslm_hip_$name.so $objs $out/slm_capi.o $base/frames.o $base/generic.o -L/opt/rocm/lib -lrccl -lrocblas -Wl,-rpath,/opt/rocm/lib
echo relinked libslm_hip_$name.so
