#!/bin/bash
# r06 session d: uint8 / CLI margin gates on the rebuilt library, then SQ counters of the complex128 radix kernels
set -o pipefail
mkdir -p gpurun_out/r06d
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread -rP tests/test_gpu_precision.py tests/test_gpu_cli.py tests/test_gpu_shuffle.py > gpurun_out/r06d/pytest_u8.log 2>&1 ;
export SLM_ENGINE=float64
timeout -k 10 600 bash tools/profile_sq.sh rz4096 --size 4096 --iters 10 --reps 1 > gpurun_out/r06d/sq4096.txt 2>&1 &&
timeout -k 10 600 bash tools/profile_sq.sh rz1024 --size 1024 --iters 20 --reps 1 > gpurun_out/r06d/sq1024.txt 2>&1
timeout -k 10 300 python -u tools/generic_speed.py --iters 20 --shapes 4096x4096 --engines rz --gd > gpurun_out/r06d/speed_cw2.txt 2>&1 &&
SLM_RZ_CW=1 timeout -k 10 300 python -u tools/generic_speed.py --iters 20 --shapes 4096x4096 --engines rz --gd > gpurun_out/r06d/speed_cw1.txt 2>&1 &&
SLM_RZ_PLAN=wide timeout -k 10 300 python -u tools/generic_speed.py --iters 20 --shapes 1024x1024 --engines rz --gd > gpurun_out/r06d/speed_1024_wide.txt 2>&1
