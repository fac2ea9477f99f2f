#!/bin/bash
# Kernel trace + PMC passes for one configuration; outputs under gpurun_out/prof_<tag>/.
# usage: tools/profile.sh <tag> <prof_gs.py args...>
set -o pipefail
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o trace -- python3 tools/prof_gs.py "$@" > $out/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o fetch -- python3 tools/prof_gs.py "$@" > $out/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -o write -- python3 tools/prof_gs.py "$@" > $out/write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d $out/sq -o sq -- python3 tools/prof_gs.py "$@" > $out/sq.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $out/tcc -o tcc -- python3 tools/prof_gs.py "$@" > $out/tcc.log 2>&1 || exit $?
echo done $tag
