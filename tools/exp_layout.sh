set -o pipefail
L=$PWD/spatial_light_modulator_module_amd/lib
for v in "" _x2y8 _x8y2; do
  echo "== lib$v"
  SLM_LIB_PATH=$L/libslm_hip$v.so timeout -k 10 100 python tools/kt.py 1024x1,1024x64,4096x1,4096x8 --precs f32 --iters 20 2>&1 | grep -v amdgpu.ids
done
SLM_LIB_PATH=$L/libslm_hip_x2y8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_gs.py tests/test_gpu_gd.py tests/test_gpu_fft.py -m gpu -q -x --timeout 600 2>&1 | tail -2
