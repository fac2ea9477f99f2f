#!/bin/bash
# r06 session c: chirp-z line transforms (rocBLAS removed) + the any-size / radix-c128 suites + 4096 gates
set -o pipefail
mkdir -p gpurun_out/r06c
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread -rP tests/test_gpu_generic.py tests/test_gpu_radix_c128.py > gpurun_out/r06c/pytest_generic.log 2>&1 ;
timeout -k 10 900 python -u -m pytest -v --timeout 800 --timeout-method thread -rP tests/test_gpu_configs.py -k "float64_engine" > gpurun_out/r06c/pytest_f64engine.log 2>&1 ;
timeout -k 10 300 python -u tools/generic_speed.py --iters 20 --shapes 97x101,1272x1024,1080x1920 --engines default,bluestein > gpurun_out/r06c/speed.txt 2>&1
