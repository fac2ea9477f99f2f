set -e
mkdir -p gpurun_out/abr
L=$PWD/spatial_light_modulator_module_amd/lib
for v in "" _rowl2 _rowl2d; do
  SLM_LIB_PATH=$L/libslm_hip$v.so timeout -k 10 120 python tools/phase_dump.py 4096 2 12 gpurun_out/abr/ph$v.sha >> gpurun_out/abr/dump.txt 2>&1
done
for pass in 1 2; do
for v in "" _rowl2 _rowl2d; do
  echo "lib $v pass $pass" >> gpurun_out/abr/kt.txt
  SLM_LIB_PATH=$L/libslm_hip$v.so timeout -k 10 180 python tools/kt.py 4096x1,4096x8 --precs f32 --iters 20 >> gpurun_out/abr/kt.txt 2>&1
done
done
for v in _rowl2 _rowl2d; do cmp -s gpurun_out/abr/ph.sha gpurun_out/abr/ph$v.sha && echo "$v bitwise equal" || echo "$v DIFFERS"; done >> gpurun_out/abr/dump.txt
mkdir -p /tmp/rp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/row_store_probe.hip -o /tmp/rp/probe && timeout -k 10 120 /tmp/rp/probe > gpurun_out/abr/probe.txt 2>&1
