#!/bin/bash
# Round-5 GPU session: $SLM_ENGINE=float64 (the any-size engine on radix-plan
# shapes): configs[2] at 500 iterations, the headline GS warm start, timing.
set -o pipefail
tag=${1:-r05p}
out=gpurun_out/$tag
mkdir -p $out
timeout -k 10 900 python -u -m pytest -v -rP --timeout 600 --timeout-method thread -m gpu -x tests/test_gpu_configs.py -k "float64_engine or configs2" > $out/pytest_f64engine.log 2>&1 || { echo "tests failed rc=$?"; tail -40 $out/pytest_f64engine.log; exit 1; }
tail -1 $out/pytest_f64engine.log
grep "\[parity\]" $out/pytest_f64engine.log
SLM_ENGINE=float64 timeout -k 10 300 python -u tools/generic_speed.py --engines mixed --shapes 1024x1024,4096x4096 --gd > $out/speed_f64engine.txt 2>&1 || { echo "speed failed"; tail $out/speed_f64engine.txt; exit 1; }
cat $out/speed_f64engine.txt
echo "done $tag"
