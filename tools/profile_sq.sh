#!/bin/bash
# Kernel trace + SQ stall counters for one configuration (separate PMC passes).
# usage: tools/profile_sq.sh <tag> <prof_gs.py args...>; outputs under gpurun_out/sq_<tag>/
set -o pipefail
tag=$1; shift
out=gpurun_out/sq_$tag
mkdir -p $out
repo=$(pwd)
cd /tmp && export TMPDIR=/tmp && cd $repo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o trace -- python3 tools/prof_gs.py "$@" > $out/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $out/sq1 -o sq1 -- python3 tools/prof_gs.py "$@" > $out/sq1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES SQ_INSTS_SALU --output-format csv -d $out/sq2 -o sq2 -- python3 tools/prof_gs.py "$@" > $out/sq2.log 2>&1 || exit $?
python3 - $out <<'PY'
import collections, csv, sys
d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for sub in ("sq1", "sq2"):
    for r in csv.DictReader(open(f"{d}/{sub}/{sub}_counter_collection.csv")):
        k = r["Kernel_Name"]
        if "_kernel<" not in k or ("col_kernel" in k and ", 0, " not in k.split("<")[1][4:9] and False):
            pass
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        if sub == "sq1" and r["Counter_Name"] == "SQ_WAVES": n[k] += 1
dur = {r["Name"]: float(r["AverageNs"]) / 1e3 for r in csv.DictReader(open(f"{d}/trace/trace_kernel_stats.csv"))}
for k, a in agg.items():
    if n[k] == 0 or a["SQ_WAVES"] == 0: continue
    w = a["SQ_WAVES"]
    wc = a["SQ_WAVE_CYCLES"]
    print(f"{k[:60]:60s} {dur.get(k, 0):8.1f}us waves/launch={w/n[k]:.0f} "
          f"valu/wave={a['SQ_INSTS_VALU']/w:.0f} lds/wave={a['SQ_INSTS_LDS']/w:.0f} "
          f"vmem_rd/wave={a['SQ_INSTS_VMEM_RD']/w:.1f} "
          f"wait_any={a['SQ_WAIT_ANY']/wc:.2f} wait_inst={a['SQ_WAIT_INST_ANY']/wc:.2f} "
          f"active={a['SQ_ACTIVE_INST_ANY']/wc:.2f} valu_active={a['SQ_ACTIVE_INST_VALU']/wc:.2f} "
          f"lds_wait={a['SQ_WAIT_INST_LDS']/wc:.3f} bankconf/lds={a['SQ_LDS_BANK_CONFLICT']/max(a['SQ_INSTS_LDS'],1):.2f} "
          f"wave_cyc={wc/w*4:.0f}")
PY
