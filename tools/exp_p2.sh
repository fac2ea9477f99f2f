set -o pipefail
L=$PWD/spatial_light_modulator_module_amd/lib
export SLM_LIB_PATH=$L/libslm_hip_p2.so
timeout -k 10 100 python tools/kt.py 1024x1,1024x64,4096x1,4096x8 --precs f32 --iters 20 2>&1 | grep -v amdgpu.ids
timeout -k 10 300 python -u -m pytest tests/test_gpu_gs.py tests/test_gpu_configs.py -m gpu -q -x --timeout 600 -k "not 4096_warm" 2>&1 | tail -2
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/p2/write -o write -- python3 tools/prof_gs.py --size 1024 --iters 20 --prec f32 > /dev/null 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/p2/fetch -o fetch -- python3 tools/prof_gs.py --size 1024 --iters 20 --prec f32 > /dev/null 2>&1 || exit 1
python3 tools/pmc_traffic.py gpurun_out/p2/fetch/fetch_counter_collection.csv gpurun_out/p2/write/write_counter_collection.csv p2_1024 gpurun_out/p2/pmc.json
