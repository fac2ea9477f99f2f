#!/bin/bash
# r06 session x: write-through stores in the last workgroups of write-back launches ($SLM_WT_TAIL),
# 4096^2 (one and eight holograms) and the 64 x 1024^2 batch, two passes
set -o pipefail
mkdir -p gpurun_out/r06x
for rep in 1 2; do
for tail in 0 512 1024 2048; do
  echo "SLM_WT_TAIL=$tail (pass $rep)"
  SLM_WT_TAIL=$tail timeout -k 10 200 python tools/kt.py 4096x1,4096x8,1024x64 --precs f32 --iters 20 || exit 1
done
done > gpurun_out/r06x/ab_wt_tail.txt 2>&1
echo "done r06x"
