set -o pipefail
out=gpurun_out/r02f; mkdir -p $out
L=$PWD/spatial_light_modulator_module_amd/lib
for v in _base ""; do
  echo "== lib$v" | tee -a $out/kt.txt
  SLM_LIB_PATH=$L/libslm_hip$v.so timeout -k 10 120 python tools/kt.py 4096x1,4096x8,2048x1,1024x1,1024x64 --precs f32 --iters 20 2>&1 | grep -v amdgpu.ids | tee -a $out/kt.txt || exit 1
  SLM_LIB_PATH=$L/libslm_hip$v.so timeout -k 10 120 python tools/phase_dump.py $out/dump$v.npz 4096x1,4096x2,2048x1,1024x1,256x3 || exit 1
done
python - <<'PY'
import numpy as np
a=np.load('gpurun_out/r02f/dump_base.npz'); b=np.load('gpurun_out/r02f/dump.npz')
for k in a.files:
    x,y=a[k],b[k]
    same=np.array_equal(x,y)
    print(f"{k:24s} bitwise {'==' if same else '!='} maxrel {np.max(np.abs(x-y)/(np.abs(x)+1e-30)):.2e}")
PY
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_gs.py -m gpu -v -rA --timeout 600 --timeout-method thread 2>&1 | grep -E "parity|PASS|FAIL|Error|passed|failed" | tail -40
