#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one counter per run, no other traces) over
# GS configurations of the bench line, reduced per launch by
# tools/pmc_traffic.py into <out>/pmc_traffic.json (merge into profiles/).
# usage: tools/pmc_configs.sh <tag> <size>:<batch>:<iters>:<prec> ...
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
repo=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd $repo
for cfg in "$@"; do
  IFS=: read -r n b it prec <<< "$cfg"
  key=gs_${n}x${n}_b${b}_it${it}_${prec}
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $out/${key}_$c -o p -- python3 tools/prof_gs.py --size $n --batch $b --iters $it --reps 1 --prec $prec > $out/${key}_$c.log 2>&1 || { echo "pass $key $c failed"; tail -5 $out/${key}_$c.log; exit 1; }
  done
  python3 tools/pmc_traffic.py $out/${key}_FETCH_SIZE/p_counter_collection.csv $out/${key}_WRITE_SIZE/p_counter_collection.csv $key $out/pmc_traffic.json > $out/${key}_traffic.txt 2>&1 || { echo "reduce $key failed"; cat $out/${key}_traffic.txt; exit 1; }
  cat $out/${key}_traffic.txt
done
echo "done $tag"
