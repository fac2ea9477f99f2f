set -o pipefail
L=$PWD/spatial_light_modulator_module_amd/lib
run() { echo "== $*"; timeout -k 10 120 env "$@" python tools/kt.py ${CFGS:-4096x1,1024x1,1024x64,2048x4} --precs f32,f64 --iters 20 --reps 2 || exit 1; }
run SLM_X=0
CFGS=4096x1 run SLM_PLAN=wide
CFGS=1024x1 run SLM_PLAN=wide SLM_COL_CW=1 SLM_LIB_PATH=$L/libslm_hip_rpw1.so
CFGS=1024x1 run SLM_PLAN=wide SLM_COL_CW=2 SLM_LIB_PATH=$L/libslm_hip_rpw2.so
CFGS=1024x1 run SLM_COL_CW=1 SLM_LIB_PATH=$L/libslm_hip_rpw1.so
CFGS=1024x64 run SLM_COL_CW=2 SLM_LIB_PATH=$L/libslm_hip_rpw2.so
