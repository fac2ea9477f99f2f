#!/bin/bash
set -o pipefail
out=gpurun_out/r05s1
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed rc=$?"; tail -30 $out/bench.err; exit 1; }
cat $out/bench.json | head -c 600
tools/pmc_ea.sh b1 --size 4096 --batch 1 --iters 40 --reps 1 > $out/ea_b1.txt 2>&1 || { cat $out/ea_b1.txt; exit 1; }
tools/pmc_ea.sh b8 --size 4096 --batch 8 --iters 40 --reps 1 > $out/ea_b8.txt 2>&1 || { cat $out/ea_b8.txt; exit 1; }
cat $out/ea_b1.txt $out/ea_b8.txt
echo done
