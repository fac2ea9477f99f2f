set -e
mkdir -p gpurun_out/s6
timeout -k 10 120 python tools/phase_dump.py 4096 2 12 gpurun_out/s6/ph.sha > gpurun_out/s6/dump.txt 2>&1
echo "digest of the r04 default build for the same run: 87689f6362f57c27ae3c44ac7de44b12ad130847c992130a5f00599305f4934c" >> gpurun_out/s6/dump.txt
timeout -k 10 240 python tools/kt.py 4096x1,4096x8 --precs f32,f64 --iters 20 > gpurun_out/s6/kt.txt 2>&1
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_gs.py tests/test_gpu_precision.py tests/test_gpu_fft.py -x -v -rP --timeout 300 --timeout-method thread > gpurun_out/s6/pytest.log 2>&1
