#!/bin/bash
# Round-5 GPU session: SQ counters of the mixed-radix engine (GS / GD 1080 x 1920).
# usage: tools/session_r05h.sh <tag>
set -o pipefail
tag=${1:-r05h}
out=gpurun_out/$tag
mkdir -p $out
tools/profile_sq.sh ${tag}_mr_gs --size 1920 --height 1080 --iters 20 --reps 1 > $out/sq_mr_gs.txt 2>&1 || { echo "sq failed"; tail -5 $out/sq_mr_gs.txt; exit 1; }
cat $out/sq_mr_gs.txt
tools/profile_sq.sh ${tag}_mr_gd --algo gd --size 1920 --height 1080 --iters 20 --reps 1 > $out/sq_mr_gd.txt 2>&1 || { echo "sq failed"; tail -5 $out/sq_mr_gd.txt; exit 1; }
cat $out/sq_mr_gd.txt
echo "done $tag"
