#!/bin/bash
# r06 session o: mixed-E complex64 plans for the 1080 / 1920 panel sides (plans.hpp ep[]) --
# panel speed against the mixed radix, the complex128 radix kernels after the position-indexed
# refactor (speed and parity), the panel parity tests, SQ counters of 1080 x 1920
set -o pipefail
mkdir -p gpurun_out/r06o
timeout -k 10 300 python -u tools/generic_speed.py --iters 50 --shapes 1080x1920,1920x1080,1200x1920,600x800,1000x1024,768x1280,1152x1536 --engines default,mr > gpurun_out/r06o/speed_c64.txt 2>&1 &&
timeout -k 10 300 python -u tools/generic_speed.py --iters 20 --shapes 4096x4096,1024x1024 --engines rz --gd > gpurun_out/r06o/speed_rz.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -rP tests/test_gpu_radix_c64.py tests/test_gpu_radix_c128.py tests/test_gpu_generic.py > gpurun_out/r06o/pytest_rz.log 2>&1 &&
timeout -k 10 600 bash tools/profile_sq.sh c64o_1080 --size 1920 --height 1080 --iters 20 --reps 1 > gpurun_out/r06o/sq_c64_1080x1920.txt 2>&1
echo "done r06o"
