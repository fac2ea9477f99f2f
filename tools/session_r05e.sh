#!/bin/bash
# Round-5 GPU session: 4096^2 correctness with whole-sector row-pair accesses,
# the bench, EA counters, the 1024^2 precision configurations, the full GPU
# suite, SQ counters of the 4096^2 batch (layout kernels included).
# usage: tools/session_r05e.sh <tag>
set -o pipefail
tag=${1:-r05e}
out=gpurun_out/$tag
mkdir -p $out
T="python -u -m pytest -v -rP --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T -x tests/test_gpu_configs.py tests/test_gpu_gs.py > $out/pytest_4096.log 2>&1 || { echo "4096 tests failed rc=$?"; tail -30 $out/pytest_4096.log; exit 1; }
tail -1 $out/pytest_4096.log
tools/gather_ab.sh $tag || { echo "gather A/B failed"; exit 1; }
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed rc=$?"; tail -30 $out/bench.err; exit 1; }
head -c 300 $out/bench.json; echo
tools/pmc_ea.sh ${tag}_b8 --size 4096 --batch 8 --iters 40 --reps 1 > $out/ea_b8.txt 2>&1 || { cat $out/ea_b8.txt; exit 1; }
tools/pmc_ea.sh ${tag}_b1 --size 4096 --batch 1 --iters 40 --reps 1 > $out/ea_b1.txt 2>&1 || { cat $out/ea_b1.txt; exit 1; }
cat $out/ea_b1.txt $out/ea_b8.txt
timeout -k 10 400 python -u tools/parity_1024.py > $out/parity_1024.txt 2>&1 || { echo "parity_1024 failed rc=$?"; tail -20 $out/parity_1024.txt; exit 1; }
cat $out/parity_1024.txt
timeout -k 10 900 $T tests > $out/pytest_gpu.log 2>&1; rc=$?; tail -3 $out/pytest_gpu.log; [ $rc -le 1 ] || { echo "pytest aborted rc=$rc"; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 $out/smoke.log; exit 1; }
tools/profile_sq.sh ${tag}_4096x8 --size 4096 --batch 8 --iters 20 --reps 1 > $out/sq_4096x8.txt 2>&1 || { echo "sq failed"; tail -5 $out/sq_4096x8.txt; exit 1; }
cat $out/sq_4096x8.txt
echo "done $tag"
