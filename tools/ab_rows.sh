#!/bin/bash
# Row-kernel A/B (tools/kt.py) at the 4096^2 and 1024^2 GS shapes over variant
# libraries: tools/ab_rows.sh <variant> ... ("" = default build), each run twice
L=spatial_light_modulator_module_amd/lib
for rep in 1 2; do
for v in "$@"; do
  so=$L/libslm_hip${v:+_$v}.so
  echo "lib ${v:-default} (pass $rep)"
  SLM_LIB_PATH=$PWD/$so python tools/kt.py 4096x1,4096x8,1024x1 --precs f32 --iters 20 || exit 1
done
done
