#!/bin/bash
# r06 session e: complex128 radix kernels after the epilogue / launder / E=8 changes -- parity, then A/B of plans
set -o pipefail
mkdir -p gpurun_out/r06e
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -rP tests/test_gpu_radix_c128.py > gpurun_out/r06e/pytest_rz.log 2>&1 &&
for rp in narrow e8; do for cp in narrow e8; do
  SLM_RZ_ROW_PLAN=$rp SLM_RZ_COL_PLAN=$cp timeout -k 10 300 python -u tools/generic_speed.py --iters 20 --shapes 4096x4096 --engines rz --gd > gpurun_out/r06e/speed_${rp}_${cp}.txt 2>&1 || exit 1
done; done
timeout -k 10 300 python -u tools/generic_speed.py --iters 40 --shapes 1024x1024,2048x2048 --engines rz --gd > gpurun_out/r06e/speed_1024.txt 2>&1 &&
SLM_ENGINE=float64 timeout -k 10 600 bash tools/profile_sq.sh rz4096e --size 4096 --iters 10 --reps 1 > gpurun_out/r06e/sq4096.txt 2>&1
