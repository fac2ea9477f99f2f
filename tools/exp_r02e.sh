set -o pipefail
mkdir -p gpurun_out/r02e
L=$PWD/spatial_light_modulator_module_amd/lib
for v in "" _pf; do
  echo "== lib$v" | tee -a gpurun_out/r02e/kt.txt
  SLM_LIB_PATH=$L/libslm_hip$v.so timeout -k 10 120 python tools/kt.py 4096x1,4096x8,2048x1 --precs f32 --iters 20 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r02e/kt.txt || exit 1
done
SLM_TRACE_BUF=1 SLM_LIB_PATH=$L/libslm_hip_pftr.so timeout -k 10 120 python tools/trace_phases.py 4096x1f32,4096x8f32 gpurun_out/r02e/trace_pf.npz 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r02e/trace_pf.txt
