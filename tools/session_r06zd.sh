#!/bin/bash
# r06 session zd: A/B of plain LDS slots after a transform's Ns >= 16 passes in the float32 engine's
# Stockham driver (4096 narrow and 1024 wide plans): kernel times (two passes) and bitwise phase digests
set -o pipefail
mkdir -p gpurun_out/r06zd
L=$PWD/spatial_light_modulator_module_amd/lib
for rep in 1 2; do for v in "" p16; do
  echo "lib ${v:-default} (pass $rep)"
  SLM_LIB_PATH=$L/libslm_hip${v:+_$v}.so timeout -k 10 200 python tools/kt.py 4096x1,4096x8,1024x64 --precs f32 --iters 20 || exit 1
done; done > gpurun_out/r06zd/ab_plain16.txt 2>&1 &&
for v in "" p16; do
  SLM_LIB_PATH=$L/libslm_hip${v:+_$v}.so timeout -k 10 200 python tools/phase_dump.py 4096 1 20 gpurun_out/r06zd/ph4096_${v:-default}.sha >> gpurun_out/r06zd/digests.txt 2>&1 || exit 1
  SLM_LIB_PATH=$L/libslm_hip${v:+_$v}.so timeout -k 10 200 python tools/phase_dump.py 1024 8 20 gpurun_out/r06zd/ph1024_${v:-default}.sha >> gpurun_out/r06zd/digests.txt 2>&1 || exit 1
done
cat gpurun_out/r06zd/*.sha >> gpurun_out/r06zd/digests.txt
echo "done r06zd"
