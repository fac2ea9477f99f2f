#!/bin/bash
# Round-5 GPU session: GD split-gradient row pass with the column maxima
# loaded first (lib/libslm_hip_lin.so) against the in-tree build.
set -o pipefail
tag=${1:-r05q}
out=gpurun_out/$tag
mkdir -p $out
NEW=$PWD/spatial_light_modulator_module_amd/lib/libslm_hip_lin.so
SLM_LIB_PATH=$NEW timeout -k 10 600 python -u -m pytest -v -rP --timeout 300 --timeout-method thread -m gpu -x tests/test_gpu_configs.py -k "gd_fused_column_pass" > $out/pytest_lin.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $out/pytest_lin.log; exit 1; }
tail -1 $out/pytest_lin.log
for rep in 1 2; do
  for lib in base new; do
    if [ $lib = new ]; then export SLM_LIB_PATH=$NEW; else unset SLM_LIB_PATH; fi
    timeout -k 10 300 python -u tools/gd_modes.py --n 1024 --modes auto,lin --check 20 > $out/gd_${lib}_$rep.txt 2>&1 || { echo "gd failed"; tail $out/gd_${lib}_$rep.txt; exit 1; }
    echo "== $lib $rep"; cut -c1-150 $out/gd_${lib}_$rep.txt
  done
done
echo "done $tag"
