#!/bin/bash
# r06 session f: complex128 radix kernels on the B2 panel layout with row pairs -- parity, then A/B of plans
set -o pipefail
mkdir -p gpurun_out/r06f
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -rP tests/test_gpu_radix_c128.py > gpurun_out/r06f/pytest_rz.log 2>&1 &&
for rp in narrow e8; do
  SLM_RZ_ROW_PLAN=$rp timeout -k 10 300 python -u tools/generic_speed.py --iters 20 --shapes 4096x4096 --engines rz --gd > gpurun_out/r06f/speed_${rp}.txt 2>&1 || exit 1
done
timeout -k 10 300 python -u tools/generic_speed.py --iters 40 --shapes 1024x1024,2048x2048 --engines rz --gd > gpurun_out/r06f/speed_1024.txt 2>&1 &&
SLM_ENGINE=float64 timeout -k 10 600 bash tools/profile_sq.sh rz4096f --size 4096 --iters 10 --reps 1 > gpurun_out/r06f/sq4096.txt 2>&1
