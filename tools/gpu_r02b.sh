#!/bin/bash
set -o pipefail
out=gpurun_out/r02b
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -m gpu -v --timeout 900 --timeout-method thread -k 4096 > $out/gate4096.log 2>&1; echo "gate rc=$?"; grep -E "parity|passed|failed" $out/gate4096.log
timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 900 --timeout-method thread --deselect tests/test_gpu_configs.py::test_gs_4096_warm_start_gate > $out/pytest_gpu.log 2>&1; rc=$?; echo "suite rc=$rc"; tail -5 $out/pytest_gpu.log; [ $rc -le 1 ] || exit 1
timeout -k 10 60 rocprofv3 -L > $out/counters.txt 2>&1 || echo "counter list rc=$?"
bash tools/profile_sq.sh r02_1024 --size 1024 --iters 20 --prec f32 || { echo "sq 1024 failed"; exit 1; }
bash tools/profile_sq.sh r02_4096 --size 4096 --iters 10 --prec f32 || { echo "sq 4096 failed"; exit 1; }
echo done
