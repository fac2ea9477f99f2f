#!/bin/bash
# Runtime-knob sweep (plan picker / store policy env overrides) over a few
# configurations, kernel times via tools/kt.py and GD structures via
# tools/gd_modes.py. usage: tools/knob_sweep.sh ; outputs on stdout.
set -o pipefail
run() { echo "## $*"; env "$@" || exit $?; }
K="python -u tools/kt.py"
run SLM_WT=1 $K 1024x64,4096x8 --precs f32 --iters 20
run SLM_WT=0 $K 1024x64,1024x1 --precs f32 --iters 20
run SLM_ROW_PLAN=narrow $K 1024x64 --precs f32 --iters 20
run SLM_COL_PLAN=narrow $K 1024x64 --precs f32 --iters 20
run SLM_COL_CW=8 $K 1024x64 --precs f32 --iters 20
run SLM_COL_CW=2 $K 1024x64 --precs f32 --iters 20
run SLM_COL_CW=4 $K 4096x8 --precs f32 --iters 20
run SLM_COL_CW=1 python -u tools/gd_modes.py --modes auto --iters 200
run SLM_COL_CW=1 $K 1024x1 --precs f32 --iters 20
