#!/bin/bash
# r06 session zh: 1920-point rows at float64 (complex128) on the 15.16.8 plan (128 threads) against 8.16.15 (240)
set -o pipefail
mkdir -p gpurun_out/r06zh
for rep in 1 2; do
  echo "default rows 8.16.15 (pass $rep)"; timeout -k 10 300 python -u tools/generic_speed.py --iters 40 --shapes 1080x1920,1200x1920 --engines rz --gd || exit 1
  echo "SLM_RZ_PANEL=main: rows 15.16.8 (pass $rep)"; SLM_RZ_PANEL=main timeout -k 10 300 python -u tools/generic_speed.py --iters 40 --shapes 1080x1920,1200x1920 --engines rz --gd || exit 1
done > gpurun_out/r06zh/ab_rows_f64.txt 2>&1
echo "done r06zh"
