#!/bin/bash
# Round-6 evidence session: the whole GPU suite, smoke, the bench line, the
# rocprofv3 kernel trace of the same bench command (frac cross-check), and the
# PMC byte passes of every bench configuration (one counter per run).
# usage: tools/session_r06_final.sh <tag> [skip-tests]
set -o pipefail
tag=${1:-r06z}
out=gpurun_out/$tag
mkdir -p $out
repo=$(pwd)
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 1500 python -u -m pytest tests -m gpu -v -rP --timeout 900 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
  tail -3 $out/pytest_gpu.log
  [ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "FAILED|Error" $out/pytest_gpu.log | head -20; }
  [ $rc -eq 0 -o $rc -eq 1 ] || exit 1   # a crash / abort / timeout ends the session
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -30 $out/smoke.log; exit 1; }
  tail -2 $out/smoke.log
fi
timeout -k 10 900 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed rc=$?"; tail -30 $out/bench.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open('$out/bench.json').read().splitlines()[-1]); print(json.dumps(d['summary']))"
cd /tmp && export TMPDIR=/tmp && cd $repo
B="bench.py --steps 5 --warmup 1 --no-extra --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o trace -- python3 $B > $out/trace.log 2>&1 || { echo "trace failed rc=$?"; tail -20 $out/trace.log; exit 1; }
python3 tools/frac_check.py $out/trace/trace_kernel_trace.csv $out/bench.json --source $tag > $out/frac_check.txt 2>&1; cat $out/frac_check.txt | tail -5
timeout -k 10 1200 bash tools/pmc_configs.sh ${tag}_pmc gs:1024:1:200:f32 gs:4096:1:200:f32 gs:4096:8:200:f32 gs:1024:64:200:f32 gd:1024:1:500:f32 gs:4096:1:200:f64:c128 gd:1024:1:500:f64:c128 gs:1080x1920:1:200:f32:radix-c64 > $out/pmc.txt 2>&1 || { echo "pmc failed"; tail -20 $out/pmc.txt; exit 1; }
echo "done $tag"
