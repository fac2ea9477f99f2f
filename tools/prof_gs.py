#!/usr/bin/env python3
"""Run one GS (or GD) configuration a few times for rocprofv3 to observe.

    python tools/prof_gs.py --size 4096 --batch 1 --iters 20 [--algo gd] [--reps 2]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatial_light_modulator_module_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--algo", default="gs")
    ap.add_argument("--u8", action="store_true")
    ap.add_argument("--prec", default="f32")  # the library default
    o = ap.parse_args()
    h = o.height or o.size
    w = o.size
    rng = np.random.default_rng(1)
    if o.u8:
        t = rng.integers(0, 256, (o.batch, h, w)).astype(np.uint8)
    else:
        t = rng.uniform(0, 255, (o.batch, h, w)).astype(np.float32)
    algo = _lib.ALGO_GD if o.algo == "gd" else _lib.ALGO_GS
    _lib.init(0)
    with _lib.Plan(algo, o.batch, h, w, _lib.TGT_U8 if o.u8 else _lib.TGT_F32, False, o.iters) as p:
        p.set_target(t)
        p.set_precision(_lib.PRECISION_F32 if o.prec == 'f32' else _lib.PRECISION_F64)
        if algo == _lib.ALGO_GD:
            p.set_lr(np.full(o.iters, 0.005, np.float32))
        for _ in range(o.reps):
            p.run(o.iters, white_attention=1.0)
        p.sync()
        print("plan", p.info())


if __name__ == "__main__":
    main()
