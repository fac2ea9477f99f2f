#!/usr/bin/env python3
"""Per-iteration time of the any-size engine's back ends next to the default
engine, GS (and GD), float32 targets, `--batch` holograms; per-kernel
HIP-event times and the physical bytes of the complex128 launches.

Engines: default (no override: float32 radix plans where the sides have one,
else the any-size engine), rz ($SLM_ENGINE=float64: the complex128 radix-plan
kernels on 2^k / 768 sides, mixed radix elsewhere), mr (the same with
$SLM_GENERIC_ENGINE=mr), bluestein ($SLM_GENERIC_ENGINE=bluestein: the
chirp-z line transforms on every side).

    python tools/generic_speed.py [--iters 50] [--shapes 1080x1920,...] [--engines default,bluestein] [--gd] [--batch 1]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatial_light_modulator_module_amd import _lib  # noqa: E402


def one(h, w, iters, algo, batch=1):
    t = np.random.default_rng(1).uniform(0, 255, (batch, h, w)).astype(np.float32)
    with _lib.Plan(algo, batch, h, w, _lib.TGT_F32, False, iters) as p:
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
    ap.add_argument("--engines", default="default,bluestein")
    ap.add_argument("--gd", action="store_true")
    ap.add_argument("--gs", type=int, default=1, help="0: GD only (with --gd)")
    ap.add_argument("--batch", type=int, default=1)
    o = ap.parse_args()
    _lib.init(0)
    algos = ([("GS", _lib.ALGO_GS)] if o.gs else []) + ([("GD", _lib.ALGO_GD)] if o.gd else [])
    for sh in o.shapes.split(","):
        h, w = (int(v) for v in sh.split("x"))
        for engine in o.engines.split(","):
            env = {"default": {}, "mixed": {}, "rz": {"SLM_ENGINE": "float64"},
                   "mr": {"SLM_ENGINE": "float64", "SLM_GENERIC_ENGINE": "mr"},
                   "bluestein": {"SLM_ENGINE": "float64", "SLM_GENERIC_ENGINE": "bluestein"}}[engine]
            for k in ("SLM_ENGINE", "SLM_GENERIC_ENGINE"):
                os.environ.pop(k, None)
            os.environ.update(env)
            for name, algo in algos:
                eng, dt, kern = one(h, w, o.iters, algo, o.batch)
                flops = 0.0
                ks = ", ".join(f"{k} {v[0]:.2f} us ({v[1]:.0f} GB/s)" for k, v in kern.items())
                print(f"{name} {o.batch}x{h}x{w} ({eng}): {dt * 1e3:.4f} ms per iteration"
                      + (f", {flops / dt / 1e12:.1f} TFLOP/s float64 in the DFT products" if flops else "")
                      + (f"; {ks}" if ks else ""), flush=True)
            if engine == "bluestein" and all(n in (768,) or n & (n - 1) == 0 for n in (h, w)):
                break  # radix-plan shape: one line is enough
    os.environ.pop("SLM_GENERIC_ENGINE", None)
    os.environ.pop("SLM_ENGINE", None)


if __name__ == "__main__":
    main()
