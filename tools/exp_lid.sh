# narrow layout pair (plan default for 1024^2 single images) against SLM_LAYOUT=default, GS and GD
set -o pipefail
for r in 1 2; do
for lay in narrow default; do
  echo "== layout $lay"
  SLM_LAYOUT=$lay timeout -k 10 100 python tools/kt.py 1024x1,1024x2 --precs f32 --iters 40 2>&1 | grep -v amdgpu.ids
  SLM_LAYOUT=$lay timeout -k 10 100 python tools/kt.py 1024x1 --precs f32 --iters 40 --algo gd 2>&1 | grep -v amdgpu.ids
done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread 2>&1 | tail -3
