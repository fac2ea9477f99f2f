#!/bin/bash
# r06 session za: twiddles of the next pass fetched before the exchange (mixed plans) --
# panel speed (complex64 and complex128) and the panel parity tests
set -o pipefail
mkdir -p gpurun_out/r06za
S=1080x1920,1920x1080,1200x1920,600x800,768x1280,1152x1536
timeout -k 10 300 python -u tools/generic_speed.py --iters 50 --shapes $S --engines default > gpurun_out/r06za/speed_c64.txt 2>&1 &&
timeout -k 10 300 python -u tools/generic_speed.py --iters 40 --shapes 1080x1920,600x800 --engines rz --gd > gpurun_out/r06za/speed_c128.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -rP tests/test_gpu_radix_c64.py tests/test_gpu_radix_c128.py > gpurun_out/r06za/pytest_rz.log 2>&1 &&
timeout -k 10 600 bash tools/profile_sq.sh c64z_1080 --size 1920 --height 1080 --iters 20 --reps 1 > gpurun_out/r06za/sq_c64_1080x1920.txt 2>&1
echo "done r06za"
