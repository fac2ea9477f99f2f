set -o pipefail
# A/B: per-launch dispatch vs HIP graph replay of the whole run (SLM_GRAPH)
run() { echo "== $*"; timeout -k 10 150 env "$@" python tools/kt.py ${CFGS:-1024x1,4096x1,1024x64,256x1} --precs f32 --iters 200 --reps 3 || exit 1; }
run SLM_GRAPH=0
run SLM_GRAPH=1
run SLM_GRAPH=0
run SLM_GRAPH=1
echo "== bench SLM_GRAPH=1"
SLM_GRAPH=1 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-extra --no-cpu-baseline 2>&1 | tail -2 || true
echo "== tests SLM_GRAPH=1"
SLM_GRAPH=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_gs.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -5
