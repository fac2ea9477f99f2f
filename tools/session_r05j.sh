#!/bin/bash
# Round-5 GPU session: mixed-radix twiddle powers (one table load per
# butterfly) against the r05 baseline build (lib/libslm_hip_mrbase.so), same
# box, alternating; the any-shape GPU tests on the new build.
# usage: tools/session_r05j.sh <tag>
set -o pipefail
tag=${1:-r05j}
out=gpurun_out/$tag
mkdir -p $out
S="1080x1920,1920x1080,1280x1024,1200x1920,1000x1000,768x1000"
for rep in 1 2; do
  for lib in base new; do
    if [ $lib = base ]; then export SLM_LIB_PATH=$PWD/spatial_light_modulator_module_amd/lib/libslm_hip_mrbase.so; else unset SLM_LIB_PATH; fi
    timeout -k 10 300 python -u tools/generic_speed.py --engines mixed --shapes $S --gd > $out/speed_${lib}_$rep.txt 2>&1 || { echo "speed $lib failed"; tail -20 $out/speed_${lib}_$rep.txt; exit 1; }
    echo "== $lib rep $rep"; cat $out/speed_${lib}_$rep.txt
  done
done
unset SLM_LIB_PATH
timeout -k 10 600 python -u -m pytest -v -rP --timeout 300 --timeout-method thread -m gpu -x tests/test_gpu_generic.py tests/test_gpu_gd.py > $out/pytest_generic.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $out/pytest_generic.log; exit 1; }
tail -1 $out/pytest_generic.log
grep "parity\|rms" $out/pytest_generic.log | head -30
echo "done $tag"
