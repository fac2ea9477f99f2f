set -o pipefail
L=$PWD/spatial_light_modulator_module_amd/lib
for v in _l2dir _l2on _col1 ""; do
  echo "== lib$v"
  SLM_LIB_PATH=$L/libslm_hip$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -k 4096 -m gpu -q -rA --timeout 600 2>&1 | grep -E "^\[parity|passed|failed"
  SLM_LIB_PATH=$L/libslm_hip$v.so timeout -k 10 100 python tools/kt.py 4096x1,4096x8 --precs f32 --iters 20 2>&1 | grep -v amdgpu.ids
done
