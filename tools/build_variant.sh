#!/bin/bash
# Build an A/B variant library: recompile only the given plan keys with extra
# flags, reuse the default build's objects for the rest.
# usage: tools/build_variant.sh <name> "<EXTRA flags>" <plan keys...>
# output: spatial_light_modulator_module_amd/lib/libslm_hip_<name>.so
set -e
name=$1; extra=$2; shift 2
root=$(cd $(dirname $0)/.. && pwd)
src=$root/spatial_light_modulator_module_amd/csrc
base=$root/build/csrc
out=$root/build/var_$name
mkdir -p $out
objs=""
for f in $base/kernels_*.o; do
  k=$(basename $f .o); k=${k#kernels_}
  if [[ " $* " == *" $k "* ]]; then objs="$objs $out/kernels_$k.o"; else objs="$objs $f"; fi
done
pids=""
for k in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=${CONTRACT:-fast} -fno-slp-vectorize -Wno-unused-function $extra -DSLM_N=$k -c $src/kernels_inst.hip -o $out/kernels_$k.o &
  pids="$pids $!"
done
# the host runtime sees the same macros (grid sizing follows tile_persistent)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=fast -fno-slp-vectorize -Wno-unused-function $extra -I/opt/rocm/include -c $src/slm_capi.hip -o $out/slm_capi.o &
pids="$pids $!"
for p in $pids; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $root/spatial_light_modulator_module_amd/lib/libslm_hip_$name.so $objs $out/slm_capi.o $base/frames.o $base/generic.o -L/opt/rocm/lib -lrccl -lrocblas -Wl,-rpath,/opt/rocm/lib
echo built libslm_hip_$name.so
