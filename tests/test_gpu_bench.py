"""bench.py's driver contract on the GPU: one short N = 1 run as a child
process (the driver runs `python bench.py` the same way) must print exactly one
JSON line with the contract's fields, a roofline object and a passing check."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_contract_n1():
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--no-extra",
           "--no-cpu-baseline"]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline"):
        assert k in out, k
    assert out["n_gpus"] == 1 and out["steps"] == 2 and out["warmup"] == 1
    assert out["unit"] == "holograms/s" and out["higher_is_better"] is True and out["scaling"] == "weak"
    assert out["dtype"] == "f32" and out["check"] == "ok" and out["value"] > 0
    assert "workload" in out["config"] and out["config"]["height"] == 1024 and out["config"]["iters"] == 200
    roof = out["roofline"]
    assert roof["bound"] == "hbm" and roof["unit"] == "GB/s" and roof["peak"] == 8000.0
    assert 0 < roof["frac"] < 1.5 and 0 < roof["frac_physical"] < 1
    assert abs(roof["frac"] - roof["achieved"] / roof["peak"]) < 1e-3
    # the step is 200 iterations of two launches: the kernels fit inside it
    assert 200 * roof["avg_us"] * 1e-3 < out["ms_per_step"]
    print(f"[bench] N=1 short run: {out['value']:.1f} holograms/s, frac {roof['frac']:.3f}")
