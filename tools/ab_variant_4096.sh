#!/bin/bash
# Generic 4096 A/B: phase digest (12 iterations, 2 x 4096^2) and kt timings of
# the default library against variant libraries libslm_hip_<name>.so.
# usage: tools/ab_variant_4096.sh <tag> <name>...
set -e
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
L=$PWD/spatial_light_modulator_module_amd/lib
for v in "" "$@"; do
  so=$L/libslm_hip${v:+_$v}.so
  SLM_LIB_PATH=$so timeout -k 10 120 python tools/phase_dump.py 4096 2 12 $out/ph_${v:-default}.sha >> $out/dump.txt 2>&1
  echo "${v:-default} $(cat $out/ph_${v:-default}.sha)" >> $out/digests.txt
done
for pass in 1 2; do
  for v in "" "$@"; do
    so=$L/libslm_hip${v:+_$v}.so
    echo "lib ${v:-default} pass $pass" >> $out/kt.txt
    SLM_LIB_PATH=$so timeout -k 10 180 python tools/kt.py 4096x1,4096x8 --precs f32 --iters 20 >> $out/kt.txt 2>&1
  done
done
