#!/bin/bash
# r02 session A: GPU suite, then SQ counters of the dominant kernels (1024^2, 4096^2).
set -o pipefail
out=gpurun_out/r02a
mkdir -p $out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $out/pytest_gpu.log; exit 1; }
tail -3 $out/pytest_gpu.log
timeout -k 10 60 rocprofv3 -L > $out/counters.txt 2>&1 || echo "counter list rc=$?"
bash tools/profile_sq.sh r02_1024 --size 1024 --iters 20 --prec f32 || { echo "sq 1024 failed"; exit 1; }
bash tools/profile_sq.sh r02_4096 --size 4096 --iters 10 --prec f32 || { echo "sq 4096 failed"; exit 1; }
echo done
