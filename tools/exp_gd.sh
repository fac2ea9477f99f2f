set -o pipefail
timeout -k 10 100 python tools/kt.py 1024x1 --precs f32 --iters 50 --algo gd 2>&1 | grep -v amdgpu.ids
timeout -k 10 100 python tools/kt.py 1024x1,4096x1 --precs f32 --iters 20 2>&1 | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest tests/test_gpu_gd.py tests/test_gpu_configs.py tests/test_gpu_stop_abi.py tests/test_gpu_gif_dtype.py tests/test_gpu_cli.py -m gpu -q -rA --timeout 600 -k "not 4096_warm" 2>&1 | grep -E "parity\] GD|passed|failed|^E " | head -20
