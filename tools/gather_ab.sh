#!/bin/bash
# A/B of the headline step with the staged comm-stream gather and r04's
# plan-stream gather; usage: tools/gather_ab.sh <tag>
set -o pipefail
out=gpurun_out/$1; mkdir -p $out
for rep in 1 2; do for g in 1 0; do
  SLM_GATHER_STAGED=$g timeout -k 10 180 python bench.py --steps 40 --warmup 3 --no-extra --no-cpu-baseline > $out/gather_ab_$g.json 2>$out/gather_ab_$g.err || { echo "bench failed"; exit 1; }
  python -c "import json; d=json.load(open('$out/gather_ab_$g.json')); r=d['ranks'][0]; print('staged=$g', d['value'], d['ms_per_step'], r['device_step_ms'], r['iteration_kernels_ms_per_run'], r['gather_ms'])"
done; done
