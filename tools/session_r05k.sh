#!/bin/bash
# Round-5 GPU session: mixed-radix column tiles of 2 / 4 forced, base vs new build.
set -o pipefail
tag=${1:-r05k}
out=gpurun_out/$tag
mkdir -p $out
S="1080x1920,1200x1920,1920x1080"
for cw in 2 4 auto; do
  for lib in base new; do
    if [ $lib = base ]; then export SLM_LIB_PATH=$PWD/spatial_light_modulator_module_amd/lib/libslm_hip_mrbase.so; else unset SLM_LIB_PATH; fi
    if [ $cw = auto ]; then unset SLM_MR_CW; else export SLM_MR_CW=$cw; fi
    timeout -k 10 300 python -u tools/generic_speed.py --engines mixed --shapes $S > $out/speed_${lib}_cw$cw.txt 2>&1 || { echo "speed failed"; tail -20 $out/speed_${lib}_cw$cw.txt; exit 1; }
    echo "== $lib cw $cw"; cat $out/speed_${lib}_cw$cw.txt
  done
done
unset SLM_MR_CW SLM_LIB_PATH
python - <<'PY'
from spatial_light_modulator_module_amd import _lib
import numpy as np
_lib.init(0)
for h, w in ((1080, 1920), (1200, 1920), (1920, 1080)):
    with _lib.Plan(_lib.ALGO_GS, 1, h, w, _lib.TGT_F32, False, 4) as p:
        print(h, w, p.info())
PY
echo "done $tag"
