#!/bin/bash
# Round-5 GPU session: mixed-radix tests and speed, the 1024^2 precision
# configurations, the GPU suite, smoke, bench, 4096^2 EA counters.
# usage: tools/session_r05d.sh <tag>
set -o pipefail
tag=${1:-r05d}
out=gpurun_out/$tag
mkdir -p $out
T="python -u -m pytest -v -rP --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T -x tests/test_gpu_generic.py > $out/pytest_generic.log 2>&1 || { echo "generic tests failed rc=$?"; tail -30 $out/pytest_generic.log; exit 1; }
tail -1 $out/pytest_generic.log
timeout -k 10 300 python -u tools/generic_speed.py --gd --engines mixed --shapes 1080x1920,1920x1080,1280x1024,1200x1920,1000x1000 > $out/generic_speed.txt 2>&1 || { echo "generic speed failed rc=$?"; tail -20 $out/generic_speed.txt; exit 1; }
cat $out/generic_speed.txt
for cw in 1 2 4; do SLM_MR_CW=$cw timeout -k 10 120 python -u tools/generic_speed.py --engines mixed --shapes 1080x1920 > $out/generic_speed_cw$cw.txt 2>&1 || { echo "cw $cw failed"; exit 1; }; echo "cw=$cw $(cat $out/generic_speed_cw$cw.txt)"; done
timeout -k 10 400 python -u tools/parity_1024.py > $out/parity_1024.txt 2>&1 || { echo "parity_1024 failed rc=$?"; tail -20 $out/parity_1024.txt; exit 1; }
cat $out/parity_1024.txt
timeout -k 10 900 $T tests > $out/pytest_gpu.log 2>&1; rc=$?; tail -3 $out/pytest_gpu.log; [ $rc -le 1 ] || { echo "pytest aborted rc=$rc"; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 $out/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed rc=$?"; tail -30 $out/bench.err; exit 1; }
head -c 400 $out/bench.json; echo
tools/pmc_ea.sh ${tag}_b1 --size 4096 --batch 1 --iters 40 --reps 1 > $out/ea_b1.txt 2>&1 || { cat $out/ea_b1.txt; exit 1; }
tools/pmc_ea.sh ${tag}_b8 --size 4096 --batch 8 --iters 40 --reps 1 > $out/ea_b8.txt 2>&1 || { cat $out/ea_b8.txt; exit 1; }
cat $out/ea_b1.txt $out/ea_b8.txt
echo "done $tag"
