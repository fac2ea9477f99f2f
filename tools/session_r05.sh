#!/bin/bash
# One round-5 GPU session: the new any-size back end first (its tests and
# speed), then the whole GPU suite, the bench and the row-pass EA counters.
# Every GPU step has its own time limit; the first failure ends the script.
# usage: tools/session_r05.sh <tag> [quick]
set -o pipefail
tag=${1:-r05}
out=gpurun_out/$tag
mkdir -p $out
T="python -u -m pytest -x -v -rP --timeout 300 --timeout-method thread"
timeout -k 10 600 $T -m gpu tests/test_gpu_generic.py tests/test_frames.py > $out/pytest_generic.log 2>&1 || { echo "generic tests failed rc=$?"; tail -40 $out/pytest_generic.log; exit 1; }
tail -2 $out/pytest_generic.log
timeout -k 10 300 python -u tools/generic_speed.py --gd > $out/generic_speed.txt 2>&1 || { echo "generic speed failed rc=$?"; tail -20 $out/generic_speed.txt; exit 1; }
cat $out/generic_speed.txt
[ "$2" = "quick" ] && exit 0
timeout -k 10 900 $T -m gpu tests > $out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $out/pytest_gpu.log; exit 1; }
tail -2 $out/pytest_gpu.log
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed rc=$?"; tail -30 $out/bench.err; exit 1; }
head -c 400 $out/bench.json; echo
tools/pmc_ea.sh ${tag}_b1 --size 4096 --batch 1 --iters 40 --reps 1 > $out/ea_b1.txt 2>&1 || { cat $out/ea_b1.txt; exit 1; }
tools/pmc_ea.sh ${tag}_b8 --size 4096 --batch 8 --iters 40 --reps 1 > $out/ea_b8.txt 2>&1 || { cat $out/ea_b8.txt; exit 1; }
cat $out/ea_b1.txt $out/ea_b8.txt
echo "done $tag"
