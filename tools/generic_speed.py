#!/usr/bin/env python3
"""Per-iteration time of the DFT-GEMM engine (image sides without a radix plan)
next to a radix-plan shape, GS, float32 targets, one hologram.

    python tools/generic_speed.py [--iters 50] [--shapes 1000x1000,1080x1920,768x1000,1024x1024]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatial_light_modulator_module_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--shapes", default="1000x1000,1080x1920,768x1000,1024x1024")
    o = ap.parse_args()
    _lib.init(0)
    for sh in o.shapes.split(","):
        h, w = (int(v) for v in sh.split("x"))
        t = np.random.default_rng(1).uniform(0, 255, (1, h, w)).astype(np.float32)
        with _lib.Plan(_lib.ALGO_GS, 1, h, w, _lib.TGT_F32, False, o.iters) as p:
            p.set_target(t)
            p.run(o.iters)
            p.sync()
            t0 = time.perf_counter()
            reps = 3
            for _ in range(reps):
                p.run(o.iters)
            p.sync()
            dt = (time.perf_counter() - t0) / reps / o.iters
            eng = p.engine()[0]
        flops = 0.0
        if eng == "dft-gemm":  # 4 complex GEMMs per iteration: 2 x (W^2 H + H^2 W) complex MACs, 8 flops each
            flops = 2 * (w * w * h + h * h * w) * 8.0
        print(f"GS {h}x{w} ({eng}): {dt * 1e3:.3f} ms per iteration"
              + (f", {flops / dt / 1e12:.1f} TFLOP/s float64 in the DFT products" if flops else ""), flush=True)


if __name__ == "__main__":
    main()
