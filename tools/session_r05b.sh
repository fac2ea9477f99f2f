#!/bin/bash
# Round-5 GPU session, second half: the GPU test files after test_gpu_gs, the
# bench and the 4096^2 row-pass EA counters. usage: tools/session_r05b.sh <tag>
set -o pipefail
tag=${1:-r05b}
out=gpurun_out/$tag
mkdir -p $out
T="python -u -m pytest -x -v -rP --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 900 $T tests/test_gpu_gs.py tests/test_gpu_multi.py tests/test_gpu_postproc.py tests/test_gpu_precision.py tests/test_gpu_shuffle.py tests/test_gpu_stop_abi.py > $out/pytest_gpu2.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $out/pytest_gpu2.log; exit 1; }
tail -2 $out/pytest_gpu2.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -20 $out/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed rc=$?"; tail -30 $out/bench.err; exit 1; }
head -c 400 $out/bench.json; echo
tools/pmc_ea.sh ${tag}_b1 --size 4096 --batch 1 --iters 40 --reps 1 > $out/ea_b1.txt 2>&1 || { cat $out/ea_b1.txt; exit 1; }
tools/pmc_ea.sh ${tag}_b8 --size 4096 --batch 8 --iters 40 --reps 1 > $out/ea_b8.txt 2>&1 || { cat $out/ea_b8.txt; exit 1; }
cat $out/ea_b1.txt $out/ea_b8.txt
echo "done $tag"
