set -o pipefail
timeout -k 10 200 python tools/kt.py 1024x1,4096x1,4096x8,1024x64,2048x4 --precs f32 --iters 20 --reps 2 || exit 1
