set -o pipefail
# Tiling/plan knobs re-checked with graph-replayed runs (1024^2 headline + small sides)
run() { echo "== $*"; timeout -k 10 150 env "$@" python tools/kt.py ${CFGS:-1024x1,512x1,2048x1} --precs f32 --iters 200 --reps 3 || exit 1; }
run SLM_X=0
run SLM_COL_CW=4
run SLM_COL_CW=1
run SLM_PLAN=wide
run SLM_PLAN=narrow
run SLM_WT=0
run SLM_WT=1
run SLM_PERSIST=2
run SLM_X=0
