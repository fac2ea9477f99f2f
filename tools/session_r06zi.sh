#!/bin/bash
# r06 session zi: radix kernels with the 1920 row plan picked per precision and algorithm -- panel / complex128 speed and parity
set -o pipefail
mkdir -p gpurun_out/r06zi
timeout -k 10 300 python -u tools/generic_speed.py --iters 50 --shapes 1080x1920,1200x1920,600x800 --engines default,rz --gd > gpurun_out/r06zi/speed.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_radix_c64.py tests/test_gpu_radix_c128.py tests/test_gpu_generic.py > gpurun_out/r06zi/pytest_rz.log 2>&1
echo "done r06zi"
