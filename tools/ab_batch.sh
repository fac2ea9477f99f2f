L=spatial_light_modulator_module_amd/lib
for rep in 1 2; do for v in "" dbl5; do so=$L/libslm_hip${v:+_$v}.so; echo "lib ${v:-default}"; SLM_LIB_PATH=$PWD/$so python tools/kt.py 1024x64,1024x16 --precs f32 --iters 20 || exit 1; done; done
