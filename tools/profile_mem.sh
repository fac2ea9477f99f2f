#!/bin/bash
# Memory-pipeline counters of one configuration, one PMC pass per block group
# (never combined with other traces); outputs under gpurun_out/mem_<tag>/.
# usage: tools/profile_mem.sh <tag> <prof_gs.py args...>
set -o pipefail
tag=$1; shift
out=gpurun_out/mem_$tag
mkdir -p $out
repo=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd $repo
i=0
for pmc in "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
           "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_WRITE_REQ_sum" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum" \
           "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAIT_ANY"; do
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
        if "_main" not in k and "kernel<" not in k: continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k][r["Counter_Name"]] += 1
for k, a in agg.items():
    c = {kk: v / n[k][kk] for kk, v in a.items()}  # per dispatch
    if c.get("SQ_WAVES", 0) < 1000: continue
    print(k[:50], " ".join(f"{kk}={v:.3g}" for kk, v in sorted(c.items())))
PY
