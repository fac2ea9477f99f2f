#!/bin/bash
# Kernel-trace A/B of variant libraries: tools/ab_variants.sh <tag> <lib.so>... ; prof_gs args from $ARGS
set -o pipefail
tag=$1; shift
for lib in "$@"; do
  n=$(basename $lib .so)
  out=gpurun_out/ab_${tag}_$n
  mkdir -p $out
  SLM_LIB_PATH=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o t -- python3 tools/prof_gs.py $ARGS > $out/log 2>&1 || { echo "FAIL $n"; exit 1; }
  python3 - $out $n <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1] + "/t_kernel_stats.csv")))
print(sys.argv[2], " | ".join(f"{r['Name'].split('<')[0].split('::')[-1]}<{r['Name'].split('<')[1][:12]} {float(r['AverageNs'])/1e3:.1f}us" for r in rows[:2]))
PY
done
