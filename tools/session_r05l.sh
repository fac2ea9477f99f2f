#!/bin/bash
# Round-5 GPU session: GD 1024^2 fused column pass with other column tiles
# (fewer barrier slots) and layouts.
set -o pipefail
tag=${1:-r05l}
out=gpurun_out/$tag
mkdir -p $out
for v in "" "SLM_LAYOUT=default" "SLM_LAYOUT=default SLM_COL_CW=4" "SLM_LAYOUT=default SLM_COL_CW=8"; do
  echo "== env: $v"
  env $v timeout -k 10 300 python -u tools/gd_modes.py --n 1024 --modes auto --check 20 > $out/gd.txt 2>&1 || { echo "gd failed"; tail -5 $out/gd.txt; exit 1; }
  cat $out/gd.txt
done
echo "done $tag"
