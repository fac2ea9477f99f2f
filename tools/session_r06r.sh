#!/bin/bash
# r06 session r: panel rows on the 8.16.15 1920 plan; A/B twiddles from global (L1/L2) instead of an LDS copy
set -o pipefail
mkdir -p gpurun_out/r06r
S=1080x1920,1920x1080,1200x1920,600x800,768x1280,1152x1536
timeout -k 10 300 python -u tools/generic_speed.py --iters 50 --shapes $S --engines default > gpurun_out/r06r/speed_c64.txt 2>&1 &&
SLM_LIB_PATH=$PWD/spatial_light_modulator_module_amd/lib/libslm_hip_twg.so timeout -k 10 300 python -u tools/generic_speed.py --iters 50 --shapes $S --engines default > gpurun_out/r06r/speed_c64_twg.txt 2>&1 &&
timeout -k 10 600 bash tools/profile_sq.sh c64r_1080 --size 1920 --height 1080 --iters 20 --reps 1 > gpurun_out/r06r/sq_c64_1080x1920.txt 2>&1
echo "done r06r"
