#!/bin/bash
# Round-5 GPU session: the 4096 narrow-8 plan (E = 8, radix 8.8.8.8, 512
# threads per line) against the shipped 16.16.16 plan: kernel times, the
# float32 +100 gate over targets 0-4, the 4096 GPU tests with the plan forced.
# usage: tools/session_r05i.sh <tag>
set -o pipefail
tag=${1:-r05i}
out=gpurun_out/$tag
mkdir -p $out
for pl in default narrow8; do
  if [ $pl = default ]; then unset SLM_PLAN; else export SLM_PLAN=$pl; fi
  timeout -k 10 300 python -u tools/kt.py 4096x1,4096x8 --precs f32 --iters 20 > $out/kt_$pl.txt 2>&1 || { echo "kt $pl failed"; tail -20 $out/kt_$pl.txt; exit 1; }
  echo "== $pl"; cat $out/kt_$pl.txt
done
unset SLM_PLAN
timeout -k 10 900 python -u tools/gate4096.py --targets 0,1,2,3,4 --plans default,narrow8 --spans 100 > $out/gate.txt 2>&1 || { echo "gate failed"; tail -30 $out/gate.txt; exit 1; }
grep -v "^RESULT" $out/gate.txt
SLM_PLAN=narrow8 timeout -k 10 600 python -u -m pytest -v -rP --timeout 300 --timeout-method thread -m gpu -x tests/test_gpu_configs.py tests/test_gpu_gs.py > $out/pytest_n8.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $out/pytest_n8.log; exit 1; }
tail -1 $out/pytest_n8.log
echo "done $tag"
