#!/bin/bash
# r06 session zb: A/B -- every radix plan of the any-size engine on the mixed-plan driver (mx_from: plain LDS
# slots after a transform's first pass, twiddles fetched ahead) against fft_core's Stockham driver
set -o pipefail
mkdir -p gpurun_out/r06zb
for v in "" mx; do
  L=$PWD/spatial_light_modulator_module_amd/lib/libslm_hip${v:+_$v}.so
  echo "lib ${v:-default}"
  SLM_LIB_PATH=$L timeout -k 10 300 python -u tools/generic_speed.py --iters 20 --shapes 4096x4096,1024x1024,2048x2048 --engines rz --gd || exit 1
  SLM_LIB_PATH=$L timeout -k 10 300 python -u tools/generic_speed.py --iters 50 --shapes 1000x1024,768x1280 --engines default || exit 1
done > gpurun_out/r06zb/ab_mx_all.txt 2>&1
echo "done r06zb"
