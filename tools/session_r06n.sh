#!/bin/bash
# r06 session n: complex64 radix kernels with LDS twiddles and per-pass address recomputation --
# speed on the panels (and the complex128 kernels the address change touches), SQ counters, then the GPU suite
set -o pipefail
mkdir -p gpurun_out/r06n
timeout -k 10 300 python -u tools/generic_speed.py --iters 50 --shapes 1080x1920,1920x1080,1200x1920,600x800,1000x1024,768x1280,1152x1536 --engines default,mr > gpurun_out/r06n/speed_c64.txt 2>&1 &&
timeout -k 10 300 python -u tools/generic_speed.py --iters 20 --shapes 4096x4096,1024x1024 --engines rz --gd > gpurun_out/r06n/speed_rz.txt 2>&1 &&
timeout -k 10 600 bash tools/profile_sq.sh c64n_1080 --size 1920 --height 1080 --iters 20 --reps 1 > gpurun_out/r06n/sq_c64_1080x1920.txt 2>&1 &&
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rP > gpurun_out/r06n/pytest_gpu.log 2>&1
echo "done r06n"
