#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one counter per run, no other traces) over
# the configurations of the bench line and its extra lines, reduced per
# launch by tools/pmc_traffic.py into <out>/pmc_traffic.json (merge into
# profiles/), each entry stamped with the plan the counters observed (the
# `plan {...}` line of tools/prof_gs.py), which bench.py checks.
# usage: tools/pmc_configs.sh <tag> <algo>:<size>[x<width>]:<batch>:<iters>:<prec>[:<engine>] ...
#   c128: $SLM_ENGINE=float64 (the complex128 radix-plan kernels; key suffix _radix-c128);
#   any other engine name (radix-c64, mixed-radix): the default plan, key suffix _<engine>
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
repo=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd $repo
for cfg in "$@"; do
  IFS=: read -r algo n b it prec eng <<< "$cfg"
  h=${n%%x*}; w=${n#*x}
  key=${algo}_${h}x${w}_b${b}_it${it}_${prec}
  envs=""
  if [ "$eng" = "c128" ]; then key=${key}_radix-c128; envs="SLM_ENGINE=float64";
  elif [ -n "$eng" ]; then key=${key}_${eng}; fi
  for c in FETCH_SIZE WRITE_SIZE; do
    if [ -n "$envs" ]; then export SLM_ENGINE=float64; else unset SLM_ENGINE; fi
    timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $out/${key}_$c -o p -- python3 tools/prof_gs.py --algo $algo --size $w --height $h --batch $b --iters $it --reps 1 --prec $prec > $out/${key}_$c.log 2>&1 || { echo "pass $key $c failed"; tail -5 $out/${key}_$c.log; exit 1; }
  done
  unset SLM_ENGINE
  python3 tools/pmc_traffic.py $out/${key}_FETCH_SIZE/p_counter_collection.csv $out/${key}_WRITE_SIZE/p_counter_collection.csv $key $out/pmc_traffic.json $out/${key}_FETCH_SIZE.log > $out/${key}_traffic.txt 2>&1 || { echo "reduce $key failed"; cat $out/${key}_traffic.txt; exit 1; }
  cat $out/${key}_traffic.txt
done
echo "done $tag"
