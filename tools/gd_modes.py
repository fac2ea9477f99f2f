#!/usr/bin/env python3
"""GD iteration structures side by side ($SLM_GD_MODE = lin | fused | two):
phase rms against the float64 oracle after `--check` iterations and per-kernel
HIP-event timing plus wall time per iteration over `--iters`.

    python tools/gd_modes.py [--n 1024] [--batch 1] [--modes lin,fused,two]
"""
import argparse
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import fast_f64, gs_gd_oracle as orc  # noqa: E402
from spatial_light_modulator_module_amd import _lib  # noqa: E402
from spatial_light_modulator_module_amd import algorithms as alg  # noqa: E402


def run(mode, t, x0, loops, timed=False):
    os.environ["SLM_GD_MODE"] = mode
    b, h, w = t.shape
    with _lib.Plan(_lib.ALGO_GD, b, h, w, _lib.TGT_F32, False, loops) as p:
        p.set_target(t)
        p.set_field(x0)
        p.set_lr(np.full(loops, 0.005, np.float32))
        p.run(loops, white_attention=1.0)
        ph, _, st, _ = p.read(expected=False)
        out = {"phase": ph, "err": st[:, :loops, 3]}
        if timed:
            us, cnt = p.run_timed(loops, white_attention=1.0)
            out["kern"] = {_lib.KERNEL_CLASS_NAMES[c]: us[c] / cnt[c] for c in range(3) if cnt[c]}
            p.sync()
            t0 = time.perf_counter()
            for _ in range(3):
                p.run(loops, white_attention=1.0)
            p.sync()
            out["wall_us"] = (time.perf_counter() - t0) / 3 / loops * 1e6
            out["info"] = p.info()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--modes", default="auto,lin,two")
    ap.add_argument("--check", type=int, default=100)
    ap.add_argument("--iters", type=int, default=500)
    o = ap.parse_args()
    _lib.init(0)
    n, b = o.n, o.batch
    t = np.stack([np.random.default_rng(1234 + k).uniform(0, 255, (n, n)).astype(np.float32) for k in range(b)])
    x0 = np.stack([alg.make_initial_guess("random", None, t[k], 42 + k) for k in range(b)])
    ref, _, ref_err, _ = fast_f64.gradient_descent_f64(t[0], o.check, 0.005, 1.0, initial_field=x0[0])
    for mode in o.modes.split(","):
        r = run(mode, t, x0, o.check)
        rms = orc.phase_rms(r["phase"][0], ref)
        erel = np.max(np.abs(r["err"][0] / ref_err - 1))
        tm = run(mode, t, x0, o.iters, timed=True)
        kern = " ".join(f"{k} {v:.2f}us" for k, v in tm["kern"].items())
        print(f"GD {b}x{n}^2 mode {mode:5s}: +{o.check} phase rms {rms:.3e} err rel {erel:.1e} | {kern} | "
              f"wall {tm['wall_us']:.2f} us/iter | {tm['info']}", flush=True)


if __name__ == "__main__":
    main()
