L=$PWD/spatial_light_modulator_module_amd/lib
for v in _col1 ""; do echo "== lib$v"; SLM_LIB_PATH=$L/libslm_hip$v.so timeout -k 10 200 python tools/diag_step.py 4096 1,2,5,20 2>&1 | grep -v amdgpu.ids; done
