#!/bin/bash
# Round-5 GPU session: swizzled relayout tiles (correctness + SQ bank
# conflicts), kernel / copy traces of the headline step with the staged and
# the plan-stream gather. usage: tools/session_r05f.sh <tag>
set -o pipefail
tag=${1:-r05f}
out=gpurun_out/$tag
mkdir -p $out
T="python -u -m pytest -v -rP --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T -x tests/test_gpu_gif_dtype.py tests/test_gpu_shuffle.py tests/test_gpu_bench.py tests/test_gpu_gs.py > $out/pytest_relayout.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $out/pytest_relayout.log; exit 1; }
tail -1 $out/pytest_relayout.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for g in 1 0; do
  SLM_GATHER_STAGED=$g timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $out/gtrace_$g -o t -- python3 bench.py --steps 8 --warmup 2 --no-extra --no-cpu-baseline > $out/gtrace_$g.json 2> $out/gtrace_$g.err || { echo "trace $g failed"; tail -20 $out/gtrace_$g.err; exit 1; }
done
tools/profile_sq.sh ${tag}_4096x8 --size 4096 --batch 8 --iters 10 --reps 1 > $out/sq_4096x8.txt 2>&1 || { echo "sq failed"; tail -5 $out/sq_4096x8.txt; exit 1; }
cat $out/sq_4096x8.txt
tools/profile_sq.sh ${tag}_1024x1 --size 1024 --batch 1 --iters 50 --reps 1 > $out/sq_1024x1.txt 2>&1 || { echo "sq failed"; tail -5 $out/sq_1024x1.txt; exit 1; }
cat $out/sq_1024x1.txt
echo "done $tag"
