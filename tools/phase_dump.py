#!/usr/bin/env python3
"""Dump GS phases / error stats of fixed configurations (for bitwise A/B of
library builds): python tools/phase_dump.py out.npz 4096x1,1024x1 [--iters 5]"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatial_light_modulator_module_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("cfgs")
    ap.add_argument("--iters", type=int, default=5)
    o = ap.parse_args()
    _lib.init(0)
    out = {}
    for cfg in o.cfgs.split(","):
        n, b = (int(v) for v in cfg.split("x"))
        rng = np.random.default_rng(n + b)
        t = rng.uniform(0, 255, (b, n, n)).astype(np.float32)
        phi = rng.uniform(-np.pi, np.pi, (b, n, n)).astype(np.float32)
        for algo in (_lib.ALGO_GS, _lib.ALGO_GD):
            with _lib.Plan(algo, b, n, n, _lib.TGT_F32, False, o.iters) as p:
                p.set_target(t)
                if algo == _lib.ALGO_GS:
                    p.set_phase(phi)
                else:
                    p.set_field(np.exp(1j * phi))
                    p.set_lr(np.full(o.iters, 0.005, np.float32))
                p.run(o.iters, white_attention=1.0)
                ph, e, st, _ = p.read()
            k = f"{'gs' if algo == _lib.ALGO_GS else 'gd'}_{cfg}"
            out[k + "_phase"], out[k + "_e"], out[k + "_err"] = ph, e, st[:, :, 3]
    np.savez(o.out, **out)


if __name__ == "__main__":
    main()
