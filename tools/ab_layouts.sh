#!/bin/bash
# 4096 layout-variant A/B (kt.py) plus the timed-run hold sweep at 1024^2
L=spatial_light_modulator_module_amd/lib
for rep in 1 2; do for v in "" "$@"; do so=$L/libslm_hip${v:+_$v}.so; echo "lib ${v:-default} (pass $rep)"; SLM_LIB_PATH=$PWD/$so python tools/kt.py 4096x1,4096x8 --precs f32 --iters 20 || exit 1; done; done
