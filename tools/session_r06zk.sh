#!/bin/bash
# r06 session zk: 1920-point complex64 columns (1920 x 1080) on 8.16.15 ($SLM_RZ_PANEL=alt) against 15.16.8
set -o pipefail
mkdir -p gpurun_out/r06zk
for rep in 1 2; do
  echo "default (pass $rep)"; timeout -k 10 300 python -u tools/generic_speed.py --iters 50 --shapes 1920x1080,1920x1920 --engines default || exit 1
  echo "SLM_RZ_PANEL=alt (pass $rep)"; SLM_RZ_PANEL=alt timeout -k 10 300 python -u tools/generic_speed.py --iters 50 --shapes 1920x1080,1920x1920 --engines default || exit 1
done > gpurun_out/r06zk/ab_cols_alt.txt 2>&1
echo "done r06zk"
