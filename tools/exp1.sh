set -o pipefail
run() { echo "== $*"; timeout -k 10 150 env "$@" python tools/kt.py ${CFGS:-4096x1,4096x8,2048x4} --precs f32 --iters 20 --reps 2 || exit 1; }
run SLM_X=0
run SLM_COL_CW=1
run SLM_COL_CW=4
