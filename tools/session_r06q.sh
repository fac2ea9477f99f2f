#!/bin/bash
# r06 session q: every 13-smooth panel plan mixed (plans.hpp ep[]), 2-column complex64 column
# tiles for 64+-thread lines; the alternative 1920 plan 8.16.15 ($SLM_RZ_PANEL=alt); panel parity
set -o pipefail
mkdir -p gpurun_out/r06q
S=1080x1920,1920x1080,1200x1920,600x800,1000x1024,768x1280,1152x1536
timeout -k 10 300 python -u tools/generic_speed.py --iters 50 --shapes $S --engines default > gpurun_out/r06q/speed_c64.txt 2>&1 &&
SLM_RZ_PANEL=alt timeout -k 10 300 python -u tools/generic_speed.py --iters 50 --shapes 1080x1920,1920x1080 --engines default > gpurun_out/r06q/speed_c64_alt.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -rP tests/test_gpu_radix_c64.py tests/test_gpu_generic.py > gpurun_out/r06q/pytest_c64.log 2>&1
echo "done r06q"
