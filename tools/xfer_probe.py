#!/usr/bin/env python3
"""Drop-in boundary transfer modes ($SLM_PIN 0/1/2 of the r04 A/B build; the shipped library copies from pageable memory):
set_target + run + read(phase) per step, host arrays in and out, at 1024^2 GS
200 iterations (bench.py's pcie_inclusive) and 4096^2 x 1 (20 iterations)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatial_light_modulator_module_amd import _lib  # noqa: E402

_lib.init(0)
for n, iters in ((1024, 200), (4096, 20)):
    t = np.random.default_rng(1234).uniform(0, 255, (1, n, n)).astype(np.float32)
    with _lib.Plan(_lib.ALGO_GS, 1, n, n, _lib.TGT_F32, False, iters) as p:
        p.set_target(t)
        p.run(iters)
        p.sync()
        t0 = time.perf_counter()
        for _ in range(5):
            p.run(iters)
        p.sync()
        dev = (time.perf_counter() - t0) / 5
        for mode in ("0", "1", "2", "0", "1", "2"):
            os.environ["SLM_PIN"] = mode
            p.set_target(t)
            p.run(iters)
            p.read(phase=True, expected=False, stats=False, iters=False)
            ts = [0.0, 0.0, 0.0]
            reps = 5
            for _ in range(reps):
                a = time.perf_counter()
                p.set_target(t)
                b = time.perf_counter()
                p.run(iters)
                p.sync()
                c = time.perf_counter()
                p.read(phase=True, expected=False, stats=False, iters=False)
                d = time.perf_counter()
                ts[0] += b - a
                ts[1] += c - b
                ts[2] += d - c
            up, run, down = (x / reps * 1e3 for x in ts)
            print(f"{n}^2 pin {mode}: set_target {up:.3f} ms, run {run:.3f} ms (device-resident {dev * 1e3:.3f}), "
                  f"read phase {down:.3f} ms, step {up + run + down:.3f} ms -> {1e3 / (up + run + down):.1f} holograms/s",
                  flush=True)
