#!/bin/bash
# r06 session v: complex128 4096^2 column tiles -- 1-column tiles (two workgroups per CU) on the
# E = 8 and E = 16 column plans against the shipped 2-column E = 8 tiles (one per CU)
set -o pipefail
mkdir -p gpurun_out/r06v
timeout -k 10 200 python -u tools/generic_speed.py --iters 20 --shapes 4096x4096 --engines rz > gpurun_out/r06v/speed_default.txt 2>&1 &&
SLM_RZ_CW=1 timeout -k 10 200 python -u tools/generic_speed.py --iters 20 --shapes 4096x4096 --engines rz > gpurun_out/r06v/speed_cw1.txt 2>&1 &&
SLM_RZ_CW=1 SLM_RZ_COL_PLAN=narrow timeout -k 10 200 python -u tools/generic_speed.py --iters 20 --shapes 4096x4096 --engines rz > gpurun_out/r06v/speed_cw1_e16.txt 2>&1 &&
SLM_RZ_CW=2 SLM_RZ_COL_PLAN=narrow timeout -k 10 200 python -u tools/generic_speed.py --iters 20 --shapes 4096x4096 --engines rz > gpurun_out/r06v/speed_cw2_e16.txt 2>&1
echo "done r06v"
