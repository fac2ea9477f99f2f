#!/bin/bash
# Round-5 GPU session: float64 GD plans with a complex128 state
# (lib/libslm_hip_f64f.so): the GD GPU tests, configs[2] precision, timing.
set -o pipefail
tag=${1:-r05o}
out=gpurun_out/$tag
mkdir -p $out
NEW=$PWD/spatial_light_modulator_module_amd/lib/libslm_hip_f64f.so
# float32 phases must be bitwise those of the in-tree build (the change only adds kernel arguments there)
for cfg in; do
  set -- $cfg
  timeout -k 10 300 python tools/phase_dump.py $1 $2 $3 $out/d_base_$1.sha > /dev/null 2>&1 || { echo "digest base failed"; exit 1; }
  SLM_LIB_PATH=$NEW timeout -k 10 300 python tools/phase_dump.py $1 $2 $3 $out/d_new_$1.sha > /dev/null 2>&1 || { echo "digest new failed"; exit 1; }
  echo "digest $cfg: base $(cat $out/d_base_$1.sha) new $(cat $out/d_new_$1.sha)"
done
export SLM_LIB_PATH=$NEW
timeout -k 10 900 python -u -m pytest -v -rP --timeout 300 --timeout-method thread -m gpu -x tests/test_gpu_gd.py tests/test_gpu_configs.py -k "gd or GD or field" > $out/pytest_gd.log 2>&1 || { echo "tests failed rc=$?"; tail -40 $out/pytest_gd.log; exit 1; }
tail -1 $out/pytest_gd.log
grep "\[parity\]" $out/pytest_gd.log
timeout -k 10 600 python -u tools/gd_precision.py --loops 100,500 > $out/gd_precision.txt 2>&1 || { echo "precision failed"; tail $out/gd_precision.txt; exit 1; }
cat $out/gd_precision.txt
timeout -k 10 300 python -u tools/kt.py 1024x1 --precs f32,f64 --algo gd --iters 50 > $out/kt_gd.txt 2>&1 || { echo "kt failed"; tail $out/kt_gd.txt; exit 1; }
cat $out/kt_gd.txt
echo "done $tag"
