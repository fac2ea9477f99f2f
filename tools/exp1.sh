set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/pt.log; exit 1; }
tail -1 gpurun_out/pt.log
for i in 1 2; do timeout -k 10 150 python tools/kt.py 4096x1,4096x8,1024x1 --precs f32 --iters 20 --reps 2 || exit 1; done
