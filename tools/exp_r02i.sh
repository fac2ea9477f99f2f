set -o pipefail
L=$PWD/spatial_light_modulator_module_amd/lib
for v in _base _col1 ""; do
  echo "== lib$v"
  SLM_LIB_PATH=$L/libslm_hip$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_configs.py -k 4096 -m gpu -q -rA --timeout 600 2>&1 | grep -E "parity|passed|failed"
done
