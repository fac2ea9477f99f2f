#!/bin/bash
# r06 session p: twiddle LDS copy behind the line loads; 2-column tiles for the complex64 panel columns
set -o pipefail
mkdir -p gpurun_out/r06p
S=1080x1920,1920x1080,1200x1920,1152x1536,768x1280
timeout -k 10 300 python -u tools/generic_speed.py --iters 50 --shapes $S --engines default > gpurun_out/r06p/speed_c64.txt 2>&1 &&
SLM_RZ_CW=2 timeout -k 10 300 python -u tools/generic_speed.py --iters 50 --shapes $S --engines default > gpurun_out/r06p/speed_c64_cw2.txt 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_radix_c64.py > gpurun_out/r06p/pytest_c64.log 2>&1
echo "done r06p"
