#!/bin/bash
# r06 session b: complex128 radix-plan back end -- parity tests, then speed vs mixed radix
set -o pipefail
mkdir -p gpurun_out/r06b
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -rP tests/test_gpu_radix_c128.py > gpurun_out/r06b/pytest_rz.log 2>&1 ;
timeout -k 10 300 python -u tools/generic_speed.py --iters 20 --shapes 4096x4096,1024x1024,768x1024 --engines rz,mr,default --gd > gpurun_out/r06b/speed.txt 2>&1 &&
timeout -k 10 300 python -u tools/parity_1024.py --u8 --seeds 1024,1025,1026 --configs f64 > gpurun_out/r06b/u8_1024_f64.txt 2>&1 &&
timeout -k 10 300 python -u tools/parity_1024.py --u8 --shape 768x1024 --seeds 21,22,23 --configs f64 > gpurun_out/r06b/u8_768_f64.txt 2>&1
