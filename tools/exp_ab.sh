# A/B timing of the default library against a variant, plus a parity subset on the default
set -o pipefail
L=$PWD/spatial_light_modulator_module_amd/lib
timeout -k 10 100 python tools/kt.py ${SHAPES:-1024x1,1024x64,4096x1,4096x8} --precs f32 --iters 20 2>&1 | grep -v amdgpu.ids
if [ -n "$VARIANT" ]; then
  echo "== $VARIANT"
  SLM_LIB_PATH=$L/libslm_hip_$VARIANT.so timeout -k 10 100 python tools/kt.py ${SHAPES:-1024x1,1024x64,4096x1,4096x8} --precs f32 --iters 20 2>&1 | grep -v amdgpu.ids
fi
if [ -n "$TRACE" ]; then
  SLM_TRACE_BUF=1 SLM_LIB_PATH=$L/libslm_hip_trace.so timeout -k 10 100 python tools/trace_phases.py $TRACE 2>&1 | grep -v amdgpu.ids
fi
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q -x --timeout 300 --timeout-method thread 2>&1 | tail -3
fi
