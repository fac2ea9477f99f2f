#!/bin/bash
# Round-5 GPU session: mixed-radix paired passes (lib/libslm_hip_pair.so)
# against the in-tree build; the any-shape tests on the paired build.
set -o pipefail
tag=${1:-r05n}
out=gpurun_out/$tag
mkdir -p $out
NEW=$PWD/spatial_light_modulator_module_amd/lib/libslm_hip_pair.so
SLM_LIB_PATH=$NEW timeout -k 10 600 python -u -m pytest -v -rP --timeout 300 --timeout-method thread -m gpu -x tests/test_gpu_generic.py > $out/pytest_pair.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $out/pytest_pair.log; exit 1; }
tail -1 $out/pytest_pair.log
S="1080x1920,1920x1080,1280x1024,1200x1920,1000x1000,768x1000"
for rep in 1 2; do
  for lib in base pair; do
    if [ $lib = pair ]; then export SLM_LIB_PATH=$NEW; else unset SLM_LIB_PATH; fi
    timeout -k 10 300 python -u tools/generic_speed.py --engines mixed --shapes $S --gd > $out/speed_${lib}_$rep.txt 2>&1 || { echo "speed failed"; tail -20 $out/speed_${lib}_$rep.txt; exit 1; }
    echo "== $lib $rep"; cat $out/speed_${lib}_$rep.txt
  done
done
echo "done $tag"
