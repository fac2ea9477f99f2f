#!/usr/bin/env python3
"""configs[2] (GD 1024^2, lr 0.005, white_attention 1, random guess seed 42,
bench target 0) at its own iteration count: phase rms against the float64
oracle for float32 and float64 butterflies (the field x is complex64 in both).

    python tools/gd_precision.py [--loops 100,500]
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import fast_f64, gs_gd_oracle as orc  # noqa: E402
from spatial_light_modulator_module_amd import _lib  # noqa: E402
from spatial_light_modulator_module_amd import algorithms as alg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--loops", default="100,500")
    ap.add_argument("--n", type=int, default=1024)
    o = ap.parse_args()
    _lib.init(0)
    n = o.n
    t = np.random.default_rng(1234).uniform(0, 255, (n, n)).astype(np.float32)
    x0 = alg.make_initial_guess("random", None, t, 42)
    for loops in (int(v) for v in o.loops.split(",")):
        ref, _, ref_err, _ = fast_f64.gradient_descent_f64(t, loops, 0.005, 1.0, initial_field=x0)
        for prec in ("f32", "f64"):
            with _lib.Plan(_lib.ALGO_GD, 1, n, n, _lib.TGT_F32, False, loops) as p:
                p.set_precision(_lib.PRECISION_F32 if prec == "f32" else _lib.PRECISION_F64)
                p.set_target(t[None])
                p.set_field(x0[None])
                p.set_lr(np.full(loops, 0.005, np.float32))
                p.run(loops, white_attention=1.0)
                ph, _, st, _ = p.read(expected=False)
            rms = orc.phase_rms(ph[0], ref)
            erel = float(np.max(np.abs(st[0, :loops, 3] / ref_err - 1)))
            print(f"GD {n}^2 {loops} iterations {prec}: phase rms {rms:.3e}  err rel {erel:.1e}", flush=True)


if __name__ == "__main__":
    main()
