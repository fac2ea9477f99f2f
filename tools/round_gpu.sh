#!/bin/bash
# One GPU-box session: GPU tests, smoke, bench, rocprofv3 kernel-trace/stats of
# the bench, and separate FETCH_SIZE / WRITE_SIZE passes (never combined with
# other traces). Every GPU step has its own time limit; the first failure ends
# the script. Outputs under gpurun_out/<tag>/.
# usage: tools/round_gpu.sh <tag> [skip-tests]
set -o pipefail
tag=${1:-r01}
out=gpurun_out/$tag
mkdir -p $out
repo=$(pwd)
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -rP --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $out/pytest_gpu.log; exit 1; }
  tail -3 $out/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed rc=$?"; tail -30 $out/smoke.log; exit 1; }
  tail -3 $out/smoke.log
fi
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed rc=$?"; tail -30 $out/bench.err; exit 1; }
cat $out/bench.json
cd /tmp && export TMPDIR=/tmp && cd $repo
B="bench.py --steps 5 --warmup 1 --no-extra --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o trace -- python3 $B > $out/trace.log 2>&1 || { echo "trace failed rc=$?"; tail -20 $out/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o fetch -- python3 $B > $out/fetch.log 2>&1 || { echo "fetch pass failed rc=$?"; tail -20 $out/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o write -- python3 $B > $out/write.log 2>&1 || { echo "write pass failed rc=$?"; tail -20 $out/write.log; exit 1; }
echo "done $tag"
