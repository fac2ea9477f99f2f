set -o pipefail
out=gpurun_out/r02h; mkdir -p $out
timeout -k 10 1500 python -u -m pytest tests -m gpu -v -rA --timeout 900 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
grep -E "^\[parity\]|FAILED|ERROR|passed|failed" $out/pytest.log | tail -60
grep -n "^E " $out/pytest.log | head -40
exit $rc
