#!/bin/bash
# r06 session u: the mixed panel plans at float64 (complex128 state: GD, uint8 GS and
# $SLM_ENGINE=float64 on SLM panels) against the float64 mixed radix; parity
set -o pipefail
mkdir -p gpurun_out/r06u
S=1080x1920,1920x1080,1200x1920,600x800,1152x1536
timeout -k 10 400 python -u tools/generic_speed.py --iters 40 --shapes $S --engines rz,mr --gd > gpurun_out/r06u/speed_c128_panels.txt 2>&1 &&
timeout -k 10 1000 python -u -m pytest -x -v --timeout 400 --timeout-method thread -rP tests/test_gpu_radix_c128.py tests/test_gpu_radix_c64.py tests/test_gpu_generic.py > gpurun_out/r06u/pytest_rz.log 2>&1
echo "done r06u"
