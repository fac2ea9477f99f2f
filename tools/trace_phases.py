#!/usr/bin/env python3
"""Per-workgroup phase timeline of the GS kernels (SLM_TRACE=1 build,
SLM_TRACE_BUF=1): where a launch's time goes (loads / transforms / stores) and
how staggered the workgroups start.

    SLM_TRACE_BUF=1 SLM_LIB_PATH=.../libslm_hip_trace.so python tools/trace_phases.py 1024x1,4096x1
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatial_light_modulator_module_amd import _lib  # noqa: E402


def summary(tr):
    t = tr.astype(np.float64) * 0.01  # 100 MHz ticks -> us
    t0 = t[:, 0].min()
    start, loads, fft, stores = t[:, 0] - t0, t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2]
    end = t[:, 3] - t0
    q = lambda a: f"{np.median(a):6.2f} [{np.percentile(a, 5):6.2f},{np.percentile(a, 95):6.2f}]"
    return (f"start {q(start)} | load {q(loads)} | fft {q(fft)} | store {q(stores)} | last end {end.max():6.2f}us "
            f"n={len(t)}")


def main():
    _lib.init(0)
    for cfg in sys.argv[1].split(","):
        prec = None
        if cfg.endswith(("f32", "f64")):
            prec = _lib.PRECISION_F32 if cfg.endswith("f32") else _lib.PRECISION_F64
            cfg = cfg[:-3]
        n, b = (int(v) for v in cfg.split("x"))
        t = np.random.default_rng(1).uniform(0, 255, (b, n, n)).astype(np.float32)
        with _lib.Plan(_lib.ALGO_GS, b, n, n, _lib.TGT_F32, False, 20) as p:
            p.set_target(t)
            if prec is not None:
                p.set_precision(prec)
            p.run(20)
            p.sync()
            for cls in (_lib.KERNEL_COL_MAIN, _lib.KERNEL_ROW_MAIN):
                print(f"{cfg:>8s} {_lib.KERNEL_CLASS_NAMES[cls]}: {summary(p.read_trace(cls))}", flush=True)


if __name__ == "__main__":
    main()
