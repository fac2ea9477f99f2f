#!/usr/bin/env python3
"""Per-workgroup timeline of the one-launch GD column pass (COL_GD_FUSED) in
an SLM_TRACE=1 build with SLM_TRACE_BUF=1: entry -> forward transform done
(slot 2) -> released by the grid max-barrier (slot 3), relative to the
earliest entry. Shows whether the barrier costs the arrival skew of the grid
or the latency of its memory-side atomics.

    SLM_TRACE_BUF=1 SLM_LIB_PATH=.../libslm_hip_trace.so python tools/trace_gd.py [size] [iters]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatial_light_modulator_module_amd import _lib  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    _lib.init(0)
    t = np.random.default_rng(1).uniform(0, 255, (1, n, n)).astype(np.float32)
    with _lib.Plan(_lib.ALGO_GD, 1, n, n, _lib.TGT_F32, False, iters) as p:
        p.set_target(t)
        p.set_lr(np.full(iters, 0.005, np.float32))
        for _ in range(3):
            p.run(iters, white_attention=1.0)
            p.sync()
        tr = p.read_trace(_lib.KERNEL_COL_MAIN).astype(np.float64)
    ent, fwd, rel = tr[:, 4] * 0.01, tr[:, 2] * 0.01, tr[:, 3] * 0.01  # 100 MHz ticks -> us
    t0 = ent.min()
    q = lambda a: f"median {np.median(a):6.2f}  p5 {np.percentile(a, 5):6.2f}  p95 {np.percentile(a, 95):6.2f}  max {a.max():6.2f}"
    print(f"GD {n}^2 last column launch, {len(ent)} workgroups (us from the first entry)")
    print("entry        ", q(ent - t0))
    print("fwd done     ", q(fwd - t0))
    print("released     ", q(rel - t0))
    print("wait         ", q(rel - fwd))
    print(f"last arrival -> first release {rel.min() - fwd.max():.2f} us, release spread {rel.max() - rel.min():.2f} us")


if __name__ == "__main__":
    main()
