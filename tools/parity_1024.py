#!/usr/bin/env python3
"""SURVEY.md 8c warm-start parity of the 1024^2 headline (30 cold float64
iterations, then +200 on the device vs the float64 oracle) on several targets,
for several arithmetic configurations of the two iteration kernels:
  f32      float32 butterflies in both (the float32 shuffle pair)
  f64      float64 butterflies in both (the float64 shuffle pair)
  col64    float64 column kernel, float32 row kernel ($SLM_ROW_PRECISION=f32)
  row64    float32 column kernel, float64 row kernel ($SLM_ROW_PRECISION=f64)
and their kernel times (HIP events).

    python tools/parity_1024.py [--seeds 1024,1234,1235] [--configs f32,f64,col64,row64]
                                [--shape 768x1024] [--u8]

--u8 draws uint8 targets (default_rng(seed).integers(0, 256)), the CLI's
input dtype (src/generate_hologram.py:102-110); --shape runs another image
shape (768x1024 is the CLI's own SLM shape).
"""
import argparse
import os
import sys

import numpy as np
import scipy.fft as sfft

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import gs_gd_oracle as orc  # noqa: E402
from spatial_light_modulator_module_amd import _lib  # noqa: E402


def run(t, phi_w, span, cfg):
    h, w = t.shape
    tt = _lib.TGT_U8 if t.dtype == np.uint8 else _lib.TGT_F32
    env = {"f32": (None, _lib.PRECISION_F32), "f64": (None, _lib.PRECISION_F64),
           "col64": ("f32", _lib.PRECISION_F64), "row64": ("f64", _lib.PRECISION_F32)}[cfg]
    if env[0]:
        os.environ["SLM_ROW_PRECISION"] = env[0]
    else:
        os.environ.pop("SLM_ROW_PRECISION", None)
    with _lib.Plan(_lib.ALGO_GS, 1, h, w, tt, False, span) as p:
        p.set_precision(env[1])  # the column kernels' (and, without the override, the rows') precision
        p.set_target(t[None])
        p.set_phase(np.asarray(phi_w, np.float32)[None])
        p.run(span)
        ph = p.read(expected=False, stats=False, iters=False)[0][0]
        us, cnt = p.run_timed(span)
        eng = p.engine()
    os.environ.pop("SLM_ROW_PRECISION", None)
    k = {_lib.KERNEL_CLASS_NAMES[c]: us[c] / cnt[c] for c in (0, 1) if cnt[c]}
    return ph, k, eng


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", default="1024,1234,1235")
    ap.add_argument("--configs", default="f32,f64,col64,row64")
    ap.add_argument("--span", type=int, default=200)
    ap.add_argument("--shape", default="1024x1024")
    ap.add_argument("--u8", action="store_true")
    o = ap.parse_args()
    _lib.init(0)
    workers = min(16, os.cpu_count() or 1)
    for seed in (int(s) for s in o.seeds.split(",")):
        h, w = (int(x) for x in o.shape.split("x"))
        rng = np.random.default_rng(seed)
        t = rng.integers(0, 256, (h, w)).astype(np.uint8) if o.u8 else rng.uniform(0, 255, (h, w)).astype(np.float32)
        with sfft.set_workers(workers):
            phi_w, _, _ = orc.gerchberg_saxton_faithful(t, 30)
            ref, _, _ = orc.gerchberg_saxton_faithful(t, o.span, initial_phase=phi_w)
        for cfg in o.configs.split(","):
            ph, k, eng = run(t, phi_w, o.span, cfg)
            print(f"{o.shape} {'u8' if o.u8 else 'f32'} seed {seed} {cfg:>6s} ({eng[0]}/{eng[1]}): phase rms {orc.phase_rms(ph, ref):.3e}; "
                  + ", ".join(f"{n} {v:.2f} us" for n, v in k.items()), flush=True)


if __name__ == "__main__":
    main()
