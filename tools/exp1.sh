set -o pipefail
# A/B of a variant library against the default build (tools/build_variant.sh)
L=$PWD/spatial_light_modulator_module_amd/lib
run() { echo "== $*"; timeout -k 10 150 env "$@" python tools/kt.py ${CFGS:-1024x1,4096x1,1024x64} --precs f32 --iters 20 --reps 2 || exit 1; }
run SLM_X=0
run SLM_LIB_PATH=$L/libslm_hip_${VARIANT:-nofence}.so
run SLM_X=0
