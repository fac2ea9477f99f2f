#!/usr/bin/env python3
"""Warm-start GS phase parity (SURVEY.md 8c protocol) of the GPU path at each
arithmetic precision, against the float64 oracle, on synthetic targets.

    python tools/precision_probe.py [--sizes 256u8,256,1024,2048] [--iters 200] [--warm 30]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from spatial_light_modulator_module_amd import _lib  # noqa: E402
from oracle import gs_gd_oracle as orc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="256u8,256,1024")
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--warm", type=int, default=30)
    ap.add_argument("--precs", default="f32,f64")
    o = ap.parse_args()
    _lib.init(0)
    for spec in o.sizes.split(","):
        u8 = spec.endswith("u8")
        n = int(spec[:-2]) if u8 else int(spec)
        rng = np.random.default_rng(2024)
        t = rng.integers(0, 256, (n, n)).astype(np.uint8) if u8 else rng.uniform(0, 255, (n, n)).astype(np.float32)
        t0 = time.time()
        phi_w, _, _ = orc.gerchberg_saxton_faithful(t, o.warm)
        ref, _, ref_err = orc.gerchberg_saxton_faithful(t, o.iters, initial_phase=phi_w)
        t_cpu = time.time() - t0
        for prec in o.precs.split(","):
            with _lib.Plan(_lib.ALGO_GS, 1, n, n, _lib.TGT_U8 if u8 else _lib.TGT_F32, False, o.iters) as p:
                p.set_precision(_lib.PRECISION_F32 if prec == "f32" else _lib.PRECISION_F64)
                p.set_target(t[None])
                p.set_phase(phi_w[None].astype(np.float32))
                p.run(o.iters)
                ph, _, st, _ = p.read(expected=False)
            rms = orc.phase_rms(ph[0], ref)
            erel = float(np.max(np.abs(st[0, :, 3] - ref_err) / np.abs(ref_err)))
            print(f"{spec:>7s} {prec} warm{o.warm}+{o.iters}: phase rms {rms:.3e}  max rel err-curve {erel:.2e}  "
                  f"(oracle {t_cpu:.0f}s)", flush=True)


if __name__ == "__main__":
    main()
