#!/bin/bash
# r06 session a: uint8 warm-start parity margins
set -o pipefail
mkdir -p gpurun_out/r06a
timeout -k 10 400 python -u tools/parity_1024.py --u8 --seeds 1024,1025,1026 --configs f32,row64 > gpurun_out/r06a/u8_1024.txt 2>&1 &&
timeout -k 10 400 python -u tools/parity_1024.py --u8 --shape 768x1024 --seeds 21,22,23 --configs f32,row64 > gpurun_out/r06a/u8_768.txt 2>&1
