#!/bin/bash
# r06 session s: the shipped panel build (mixed plans, 8.16.15 rows of 1920, table twiddles): speed + parity
set -o pipefail
mkdir -p gpurun_out/r06s
S=1080x1920,1920x1080,1200x1920,600x800,1000x1024,768x1280,1152x1536
timeout -k 10 300 python -u tools/generic_speed.py --iters 50 --shapes $S --engines default,mr > gpurun_out/r06s/speed_c64.txt 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -rP tests/test_gpu_radix_c64.py tests/test_gpu_generic.py tests/test_gpu_radix_c128.py > gpurun_out/r06s/pytest_rz.log 2>&1
echo "done r06s"
