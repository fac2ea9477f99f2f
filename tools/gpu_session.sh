#!/bin/bash
# One ad-hoc GPU session: each step under its own time limit, the first
# failure ends the script. usage: tools/gpu_session.sh <tag> "<step>" ["<step>" ...]
# A step is a shell command line; its output goes to gpurun_out/<tag>/<n>.log.
set -o pipefail
tag=$1; shift
out=gpurun_out/$tag
mkdir -p $out
n=0
for step in "$@"; do
  n=$((n + 1))
  echo "== step $n: $step" | tee -a $out/steps.txt
  timeout -k 10 ${STEP_TIMEOUT:-300} bash -c "$step" > $out/$n.log 2>&1
  rc=$?
  tail -${TAIL:-15} $out/$n.log
  if [ $rc -ne 0 ]; then echo "step $n failed rc=$rc"; exit $rc; fi
done
echo "session $tag done"
