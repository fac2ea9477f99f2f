#!/usr/bin/env python3
"""Per-workgroup phase timeline of the GS kernels (SLM_TRACE=1 build,
SLM_TRACE_BUF=1): where a launch's time goes (entry -> loads issued ->
loads done -> transforms -> stores) and how many workgroups each CU really
holds at once.

    SLM_TRACE_BUF=1 SLM_LIB_PATH=.../libslm_hip_trace.so python tools/trace_phases.py 1024x1,4096x1 [out.npz]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatial_light_modulator_module_amd import _lib  # noqa: E402


def summary(tr):
    t = tr[:, :5].astype(np.float64) * 0.01  # 100 MHz ticks -> us
    t0 = t[:, 4].min()
    entry = t[:, 4] - t0
    issue, loads, fft, stores = t[:, 0] - t[:, 4], t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2]
    end = t[:, 3] - t0
    q = lambda a: f"{np.median(a):6.2f} [{np.percentile(a, 5):6.2f},{np.percentile(a, 95):6.2f}]"
    # concurrency: workgroups alive per CU (HW_ID cu/sh/se + XCC id) over time
    hw = tr[:, 5].astype(np.int64)
    cu_key = (tr[:, 6].astype(np.int64) & 0xF) * 4096 + ((hw >> 8) & 0x1FF)
    keys, inv = np.unique(cu_key, return_inverse=True)
    span = end.max()
    busy = np.zeros(len(keys))
    np.add.at(busy, inv, end - entry)
    conc = busy / span
    # peak concurrency per CU by sweep
    peak = []
    for k in range(len(keys)):
        sel = inv == k
        ev = sorted([(a, 1) for a in entry[sel]] + [(b, -1) for b in end[sel]])
        c = m = 0
        for _, d in ev:
            c += d
            m = max(m, c)
        peak.append(m)
    return (f"entry {q(entry)} | issue {q(issue)} | load {q(loads)} | fft {q(fft)} | store {q(stores)} | "
            f"last end {span:6.2f}us n={len(t)} | CUs {len(keys)} wg/CU avg {np.mean(conc):4.2f} "
            f"peak {np.median(peak):.0f} [{np.min(peak)},{np.max(peak)}]")


def main():
    _lib.init(0)
    dump = {}
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
                tr = p.read_trace(cls)
                dump[f"{cfg}_{_lib.KERNEL_CLASS_NAMES[cls]}"] = tr
                print(f"{cfg:>8s} {_lib.KERNEL_CLASS_NAMES[cls]}: {summary(tr)}", flush=True)
    if len(sys.argv) > 2:
        np.savez_compressed(sys.argv[2], **dump)


if __name__ == "__main__":
    main()
