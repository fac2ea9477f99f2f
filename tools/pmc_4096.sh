#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one counter group per run, no other traces)
# over the 4096^2 GS configurations of the bench's extra lines, reduced per
# launch by tools/pmc_traffic.py into profiles/pmc_traffic.json.
# usage: tools/pmc_4096.sh <tag>
set -o pipefail
tag=${1:-pmc4096}
out=gpurun_out/$tag
mkdir -p $out
repo=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd $repo
for b in 1 8; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $out/b${b}_$c -o p -- python3 tools/prof_gs.py --size 4096 --batch $b --iters 200 --reps 1 > $out/b${b}_$c.log 2>&1 || { echo "pass b$b $c failed"; tail -5 $out/b${b}_$c.log; exit 1; }
  done
  python3 tools/pmc_traffic.py $out/b${b}_FETCH_SIZE/p_counter_collection.csv $out/b${b}_WRITE_SIZE/p_counter_collection.csv gs_4096x4096_b${b}_it200_f32 $out/pmc_traffic.json > $out/b${b}_traffic.txt 2>&1 || { echo "reduce b$b failed"; cat $out/b${b}_traffic.txt; exit 1; }
done
echo "done $tag"
