#!/usr/bin/env python3
"""Per-iteration time of the any-size engine's two back ends (mixed radix and
DFT-GEMM, image sides without a float32 radix plan) next to a radix-plan
shape, GS (and GD), float32 targets, one hologram; per-kernel HIP-event times
and the physical bytes of the mixed-radix launches.

    python tools/generic_speed.py [--iters 50] [--shapes 1080x1920,...] [--engines mixed,gemm] [--gd]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatial_light_modulator_module_amd import _lib  # noqa: E402


def one(h, w, iters, algo):
    t = np.random.default_rng(1).uniform(0, 255, (1, h, w)).astype(np.float32)
    with _lib.Plan(algo, 1, h, w, _lib.TGT_F32, False, iters) as p:
        p.set_target(t)
        wa = 0.0
        if algo == _lib.ALGO_GD:
            p.set_lr(np.full(iters, 0.005, np.float32))
            wa = 1.0
        p.run(iters, white_attention=wa)
        p.sync()
        t0 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            p.run(iters, white_attention=wa)
        p.sync()
        dt = (time.perf_counter() - t0) / reps / iters
        eng = p.engine()[0]
        us, cnt = p.run_timed(iters, white_attention=wa)
        kern = {}
        for cls in (_lib.KERNEL_COL_MAIN, _lib.KERNEL_ROW_MAIN, _lib.KERNEL_GD_STATS):
            if cnt[cls]:
                avg = us[cls] / cnt[cls]
                b = p.kernel_bytes(cls)
                kern[_lib.KERNEL_CLASS_NAMES[cls]] = (avg, b / (avg * 1e-6) / 1e9 if b else 0.0)
    return eng, dt, kern


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--shapes", default="1080x1920,1920x1080,1280x1024,1200x1920,1000x1000,768x1000,1024x1024")
    ap.add_argument("--engines", default="mixed,gemm")
    ap.add_argument("--gd", action="store_true")
    o = ap.parse_args()
    _lib.init(0)
    algos = [("GS", _lib.ALGO_GS)] + ([("GD", _lib.ALGO_GD)] if o.gd else [])
    for sh in o.shapes.split(","):
        h, w = (int(v) for v in sh.split("x"))
        for engine in o.engines.split(","):
            if engine == "gemm":
                os.environ["SLM_GENERIC_ENGINE"] = "gemm"
            else:
                os.environ.pop("SLM_GENERIC_ENGINE", None)
            for name, algo in algos:
                eng, dt, kern = one(h, w, o.iters, algo)
                flops = 2 * (w * w * h + h * h * w) * 8.0 if eng == "dft-gemm" else 0.0
                ks = ", ".join(f"{k} {v[0]:.2f} us ({v[1]:.0f} GB/s)" for k, v in kern.items())
                print(f"{name} {h}x{w} ({eng}): {dt * 1e3:.4f} ms per iteration"
                      + (f", {flops / dt / 1e12:.1f} TFLOP/s float64 in the DFT products" if flops else "")
                      + (f"; {ks}" if ks else ""), flush=True)
            if engine == "gemm" and all(n in (768,) or n & (n - 1) == 0 for n in (h, w)):
                break  # radix-plan shape: one line is enough
    os.environ.pop("SLM_GENERIC_ENGINE", None)


if __name__ == "__main__":
    main()
