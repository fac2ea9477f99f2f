#!/bin/bash
# r06 session zj: complex64 1920-point panel rows under a 6-waves-per-SIMD register floor (three 480-thread
# row-pair tiles per CU: a 1080-row panel in one round) -- speed and the complex64 parity tests
set -o pipefail
mkdir -p gpurun_out/r06zj
timeout -k 10 300 python -u tools/generic_speed.py --iters 50 --shapes 1080x1920,1200x1920,1920x1920 --engines default > gpurun_out/r06zj/speed.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_radix_c64.py > gpurun_out/r06zj/pytest_c64.log 2>&1
echo "done r06zj"
