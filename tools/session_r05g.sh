#!/bin/bash
# Round-5 GPU session: relayout + gather tests, the 4096^2 phase digest
# against r04's, gather A/B, the bench and its rocprofv3 kernel trace, PMC
# traffic of the bench's GS configurations, SQ of 1024^2, GD modes.
# usage: tools/session_r05g.sh <tag>
set -o pipefail
tag=${1:-r05g}
out=gpurun_out/$tag
mkdir -p $out
repo=$(pwd)
T="python -u -m pytest -v -rP --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T -x tests/test_gpu_gif_dtype.py tests/test_gpu_shuffle.py tests/test_gpu_bench.py tests/test_gpu_multi.py tests/test_gpu_gs.py > $out/pytest_part.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $out/pytest_part.log; exit 1; }
tail -1 $out/pytest_part.log
timeout -k 10 300 python tools/phase_dump.py 4096 2 12 $out/digest_4096.sha > $out/digest.log 2>&1 || { echo "digest failed"; tail $out/digest.log; exit 1; }
echo "digest $(cat $out/digest_4096.sha) (r04: 87689f6362f57c27ae3c44ac7de44b12ad130847c992130a5f00599305f4934c)"
tools/gather_ab.sh $tag || { echo "gather A/B failed"; exit 1; }
timeout -k 10 600 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed rc=$?"; tail -30 $out/bench.err; exit 1; }
head -c 400 $out/bench.json; echo
cd /tmp && export TMPDIR=/tmp && cd $repo
B="bench.py --steps 5 --warmup 1 --no-extra --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o trace -- python3 $B > $out/trace.json 2> $out/trace.log || { echo "trace failed rc=$?"; tail -20 $out/trace.log; exit 1; }
tools/pmc_configs.sh ${tag}_pmc 4096:1:200:f32 4096:8:200:f32 1024:1:200:f32 > $out/pmc.txt 2>&1 || { echo "pmc failed"; tail -5 $out/pmc.txt; exit 1; }
cat $out/pmc.txt
tools/profile_sq.sh ${tag}_1024x1 --size 1024 --batch 1 --iters 50 --reps 1 > $out/sq_1024x1.txt 2>&1 || { echo "sq failed"; tail -5 $out/sq_1024x1.txt; exit 1; }
cat $out/sq_1024x1.txt
timeout -k 10 300 python -u tools/gd_modes.py --n 1024 > $out/gd_modes.txt 2>&1 || { echo "gd modes failed"; tail -20 $out/gd_modes.txt; exit 1; }
cat $out/gd_modes.txt
echo "done $tag"
