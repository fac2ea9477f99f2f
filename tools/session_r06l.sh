#!/bin/bash
# r06 session l: complex64 radix kernels on 13-smooth panels -- parity, speed against the mixed radix, SQ counters
set -o pipefail
mkdir -p gpurun_out/r06l
timeout -k 10 300 python -u tools/generic_speed.py --iters 50 --shapes 1080x1920,1920x1080,1200x1920,600x800,1000x1024,768x1280,1152x1536 --engines default,mr > gpurun_out/r06l/speed_c64.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -rP tests/test_gpu_radix_c64.py tests/test_gpu_generic.py > gpurun_out/r06l/pytest_c64.log 2>&1 &&
timeout -k 10 600 bash tools/profile_sq.sh c64_1080 --size 1920 --height 1080 --iters 20 --reps 1 > gpurun_out/r06l/sq_c64_1080.txt 2>&1 &&
timeout -k 10 600 bash tools/pmc_configs.sh r06l_pmc gs:1080x1920:1:200:f32:radix-c64 > gpurun_out/r06l/pmc.txt 2>&1
echo "done r06l"
