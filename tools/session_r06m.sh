#!/bin/bash
# r06 session m: complex64 radix kernels -- SQ counters of the panel passes, then parity
set -o pipefail
mkdir -p gpurun_out/r06m
timeout -k 10 600 bash tools/profile_sq.sh c64_1080 --size 1920 --height 1080 --iters 20 --reps 1 > gpurun_out/r06m/sq_c64_1080x1920.txt 2>&1 &&
timeout -k 10 600 bash tools/profile_sq.sh c64_1920 --size 1080 --height 1920 --iters 20 --reps 1 > gpurun_out/r06m/sq_c64_1920x1080.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -rP tests/test_gpu_radix_c64.py tests/test_gpu_generic.py > gpurun_out/r06m/pytest_c64.log 2>&1
echo "done r06m"
