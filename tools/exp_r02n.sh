set -o pipefail
timeout -k 10 100 python tools/kt.py 1024x1,4096x1,4096x8,1024x64 --precs f32 --iters 20 2>&1 | grep -v amdgpu.ids
timeout -k 10 100 python tools/kt.py 1024x1 --precs f32 --iters 50 --algo gd 2>&1 | grep -v amdgpu.ids
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 900 --timeout-method thread 2>&1 | tail -3
