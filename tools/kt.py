#!/usr/bin/env python3
"""Per-kernel-class timing (HIP events on the plan stream) of GS/GD plans over
a list of configurations and precisions, for quick A/B runs on the GPU box.

    python tools/kt.py 1024x1,4096x1,1024x64 [--precs f32,f64] [--iters 20] [--algo gs]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatial_light_modulator_module_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cfgs", default="1024x1,4096x1")
    ap.add_argument("--precs", default="f64")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--algo", default="gs")
    ap.add_argument("--reps", type=int, default=3)
    o = ap.parse_args()
    _lib.init(0)
    algo = _lib.ALGO_GD if o.algo == "gd" else _lib.ALGO_GS
    for cfg in o.cfgs.split(","):
        n, b = (int(v) for v in cfg.split("x"))
        t = np.random.default_rng(1).uniform(0, 255, (b, n, n)).astype(np.float32)
        with _lib.Plan(algo, b, n, n, _lib.TGT_F32, False, o.iters) as p:
            p.set_target(t)
            if algo == _lib.ALGO_GD:
                p.set_lr(np.full(o.iters, 0.005, np.float32))
            for prec in o.precs.split(","):
                p.set_precision(_lib.PRECISION_F32 if prec == "f32" else _lib.PRECISION_F64)
                p.run(o.iters, white_attention=1.0)
                p.sync()
                us, cnt = p.run_timed(o.iters, white_attention=1.0)
                parts = []
                tot = 0.0
                for c in range(_lib.NUM_KERNEL_CLASSES - 1):
                    if cnt[c]:
                        a = us[c] / cnt[c]
                        gbs = p.kernel_bytes(c) / (a * 1e-6) / 1e9
                        parts.append(f"{_lib.KERNEL_CLASS_NAMES[c]} {a:8.2f}us {gbs:7.0f}GB/s")
                        tot += a
                import time
                p.sync()
                t0 = time.perf_counter()
                for _ in range(o.reps):
                    p.run(o.iters, white_attention=1.0)
                p.sync()
                wall = (time.perf_counter() - t0) / o.reps / o.iters * 1e6
                info = p.info()
                tiles = f"cw{info['col_cw']} rpw{info['rows_per_workgroup']} plans {info['col_plan']}/{info['row_plan']}"
                print(f"{cfg:>10s} {prec} {o.algo}: " + " | ".join(parts) + f" | kernels {tot:8.2f}us "
                      f"wall {wall:8.2f}us/iter ({wall / b:.2f}us/holo) {tiles}", flush=True)


if __name__ == "__main__":
    main()
