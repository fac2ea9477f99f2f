set -o pipefail
L=$PWD/spatial_light_modulator_module_amd/lib
run() { echo "== $*"; timeout -k 10 150 env "$@" python tools/kt.py ${CFGS:-4096x1,1024x1,1024x64,2048x4} --precs f32 --iters 20 --reps 2 || exit 1; }
run SLM_X=0
run SLM_LIB_PATH=$L/libslm_hip_rowpow.so
run SLM_LIB_PATH=$L/libslm_hip_rowchain.so
