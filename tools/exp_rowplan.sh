set -o pipefail
# Row-pass radix plan chosen separately from the column pass (SLM_ROW_PLAN)
run() { echo "== $*"; timeout -k 10 150 env "$@" python tools/kt.py ${CFGS:-2048x1,2048x4,2048x16,1024x1,1024x8,1024x64,512x1} --precs f32 --iters 100 --reps 3 || exit 1; }
run SLM_X=0
run SLM_ROW_PLAN=narrow
run SLM_ROW_PLAN=wide
run SLM_X=0
run SLM_ROW_PLAN=narrow
