set -o pipefail
out=gpurun_out/r02g; mkdir -p $out
timeout -k 10 120 python tools/kt.py 4096x1,4096x8,2048x1,1024x1,1024x64 --precs f32 --iters 20 2>&1 | grep -v amdgpu.ids | tee $out/kt.txt || exit 1
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -rA --timeout 900 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
grep -E "^\[parity\]|PASSED|FAILED|ERROR|passed|failed" $out/pytest.log | grep -v "^PASSED" | tail -60
exit $rc
