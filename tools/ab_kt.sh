#!/bin/bash
# Kernel-class timing A/B of variant libraries (tools/kt.py, HIP events) on the
# headline GS and the GD 1024^2 plans: tools/ab_kt.sh <variant> ... ("" = default build)
L=spatial_light_modulator_module_amd/lib
for v in "$@"; do
  so=$L/libslm_hip${v:+_$v}.so
  echo "lib ${v:-default}"
  SLM_LIB_PATH=$PWD/$so python tools/kt.py 1024x1 --precs f32 --iters 200 || exit 1
  SLM_LIB_PATH=$PWD/$so python tools/kt.py 1024x1 --precs f32 --iters 200 --algo gd || exit 1
done
