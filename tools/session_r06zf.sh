#!/bin/bash
# r06 session zf: complex64 panel column tiles of 4 columns (LDS now holds no twiddles) against the shipped 2
set -o pipefail
mkdir -p gpurun_out/r06zf
S=1080x1920,1920x1080,1200x1920,1152x1536,768x1280
for rep in 1 2; do
  echo "default (pass $rep)"; timeout -k 10 300 python -u tools/generic_speed.py --iters 50 --shapes $S --engines default || exit 1
  echo "SLM_RZ_CW=4 (pass $rep)"; SLM_RZ_CW=4 timeout -k 10 300 python -u tools/generic_speed.py --iters 50 --shapes $S --engines default || exit 1
done > gpurun_out/r06zf/ab_cw4.txt 2>&1
echo "done r06zf"
