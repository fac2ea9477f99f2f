#!/bin/bash
# A/B of the packed butterfly additions (-DSLM_PK=1, plan key 13 = float32 4096
# narrow): phase digest against the default build, then kernel timings.
set -e
mkdir -p gpurun_out/abpk
L=$PWD/spatial_light_modulator_module_amd/lib
for v in "" _pk; do
  SLM_LIB_PATH=$L/libslm_hip$v.so timeout -k 10 120 python tools/phase_dump.py 4096 2 12 gpurun_out/abpk/ph$v.sha >> gpurun_out/abpk/dump.txt 2>&1
done
for pass in 1 2; do
for v in "" _pk; do
  echo "lib $v pass $pass" >> gpurun_out/abpk/kt.txt
  SLM_LIB_PATH=$L/libslm_hip$v.so timeout -k 10 180 python tools/kt.py 4096x1,4096x8 --precs f32 --iters 20 >> gpurun_out/abpk/kt.txt 2>&1
done
done
