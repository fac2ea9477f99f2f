#!/bin/bash
# Round-5 GPU session: 4096 row pairs with the bank-masked DPP half-sector swap
# (lib/libslm_hip_swap.so) against the in-tree build: phase digest (must be
# bitwise equal) and kernel times, alternating.
set -o pipefail
tag=${1:-r05m}
out=gpurun_out/$tag
mkdir -p $out
NEW=$PWD/spatial_light_modulator_module_amd/lib/libslm_hip_swap.so
SLM_LIB_PATH=$NEW timeout -k 10 300 python tools/phase_dump.py 4096 2 12 $out/digest_swap.sha > $out/digest.log 2>&1 || { echo "digest failed"; tail $out/digest.log; exit 1; }
echo "digest swap $(cat $out/digest_swap.sha) (r04/r05: 87689f6362f57c27ae3c44ac7de44b12ad130847c992130a5f00599305f4934c)"
for rep in 1 2; do
  for lib in base swap; do
    if [ $lib = swap ]; then export SLM_LIB_PATH=$NEW; else unset SLM_LIB_PATH; fi
    timeout -k 10 300 python -u tools/kt.py 4096x1,4096x8 --precs f32 --iters 20 > $out/kt_${lib}_$rep.txt 2>&1 || { echo "kt failed"; tail -20 $out/kt_${lib}_$rep.txt; exit 1; }
    echo "== $lib $rep"; cat $out/kt_${lib}_$rep.txt
  done
done
echo "done $tag"
