#!/bin/bash
# L2 -> fabric request sizes (TCC_EA0_*) per launch of one configuration: how
# many write requests leave L2 as 64-B pieces and reads as 32-B pieces (partial
# lines that did not merge in L2). One PMC pass per counter pair, no other
# traces. usage: tools/pmc_ea.sh <tag> <prof_gs.py args...>
set -o pipefail
tag=$1; shift
out=gpurun_out/ea_$tag
mkdir -p $out
repo=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd $repo
i=0
for pmc in "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d $out/p$i -o p$i -- python3 tools/prof_gs.py "$@" > $out/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $out/p$i.log; exit 1; }
done
python3 - $out <<'PY'
import collections, csv, glob, sys
d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(collections.Counter)
for f in glob.glob(f"{d}/p*/p*_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "row_kernel" not in k and "col_kernel" not in k: continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k][r["Counter_Name"]] += 1
for k, a in sorted(agg.items()):
    c = {kk: v / n[k][kk] for kk, v in a.items()}  # per dispatch
    if min(n[k].values()) < 20: continue
    print(k[:60], " ".join(f"{kk}={v:.4g}" for kk, v in sorted(c.items())))
PY
