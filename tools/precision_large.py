#!/usr/bin/env python3
"""Warm-start GS phase parity at large sizes (SURVEY.md 8c protocol) with
checkpoints: the float64 oracle continues phi_warm by 50, 100, 200 iterations
(scipy.fft over many host threads: pocketfft's per-line transforms are the same
bits at any thread count) and the GPU runs the same spans from phi_warm at each
precision.

    python tools/precision_large.py --n 4096 [--u8] [--spans 50,100,200] [--workers 32]
"""
import argparse
import os
import sys
import time

import numpy as np
import scipy.fft as sfft

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from spatial_light_modulator_module_amd import _lib  # noqa: E402
from oracle import gs_gd_oracle as orc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--warm", type=int, default=30)
    ap.add_argument("--spans", default="50,100,200")
    ap.add_argument("--precs", default="f64,f32")
    ap.add_argument("--workers", type=int, default=32)
    ap.add_argument("--u8", action="store_true")
    o = ap.parse_args()
    n = o.n
    rng = np.random.default_rng(2024)
    t = rng.integers(0, 256, (n, n)).astype(np.uint8) if o.u8 else rng.uniform(0, 255, (n, n)).astype(np.float32)
    spans = [int(s) for s in o.spans.split(",")]
    t0 = time.time()
    with sfft.set_workers(o.workers):
        phi_w, _, _ = orc.gerchberg_saxton_faithful(t, o.warm)
        refs = {}
        phi, done = phi_w, 0
        for s in spans:
            phi, _, _ = orc.gerchberg_saxton_faithful(t, s - done, initial_phase=phi)
            done = s
            refs[s] = phi
            print(f"oracle +{s} at {time.time() - t0:.0f}s", flush=True)
    print(f"oracle {n}x{n} warm {o.warm} + {spans[-1]}: {time.time() - t0:.0f}s", flush=True)
    _lib.init(0)
    for prec in o.precs.split(","):
        with _lib.Plan(_lib.ALGO_GS, 1, n, n, _lib.TGT_U8 if o.u8 else _lib.TGT_F32, False, spans[-1]) as p:
            p.set_precision(_lib.PRECISION_F32 if prec == "f32" else _lib.PRECISION_F64)
            p.set_target(t[None])
            out = []
            for s in spans:
                p.set_phase(phi_w[None].astype(np.float32))
                p.run(s)
                ph, _, _, _ = p.read(expected=False)
                out.append(f"+{s}: {orc.phase_rms(ph[0], refs[s]):.3e}")
        print(f"{n}{'u8' if o.u8 else ''} {prec}: " + "  ".join(out), flush=True)


if __name__ == "__main__":
    main()
