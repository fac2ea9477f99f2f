#!/bin/bash
# r06 session zc: every radix plan on the mixed-plan driver -- speed and the radix-engine parity tests,
# including configs[4] at 200 and configs[2] at 500 on the complex128 engine
set -o pipefail
mkdir -p gpurun_out/r06zc
timeout -k 10 300 python -u tools/generic_speed.py --iters 20 --shapes 4096x4096,1024x1024 --engines rz --gd > gpurun_out/r06zc/speed_rz.txt 2>&1 &&
timeout -k 10 300 python -u tools/generic_speed.py --iters 50 --shapes 1080x1920,1920x1080,1000x1024,768x1280 --engines default > gpurun_out/r06zc/speed_c64.txt 2>&1 &&
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -rP tests/test_gpu_radix_c128.py tests/test_gpu_radix_c64.py tests/test_gpu_generic.py tests/test_gpu_configs.py -k "radix or generic or float64_engine or c64 or c128" > gpurun_out/r06zc/pytest_rz.log 2>&1
echo "done r06zc"
