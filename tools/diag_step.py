#!/usr/bin/env python3
"""Per-step GS precision vs the float64 oracle from a warmed state:
python tools/diag_step.py 4096 [1,2,5,20]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import fast_f64, gs_gd_oracle as orc  # noqa: E402
from spatial_light_modulator_module_amd import _lib  # noqa: E402


def main():
    n = int(sys.argv[1])
    steps = [int(s) for s in (sys.argv[2] if len(sys.argv) > 2 else "1,2,5,20").split(",")]
    _lib.init(0)
    t = np.random.default_rng(1234).uniform(0, 255, (n, n)).astype(np.float32)
    phi30, _, _ = fast_f64.gerchberg_saxton_f64(t, 30)
    phi30 = phi30.astype(np.float32)
    for s in steps:
        ref, e_ref, err_ref = fast_f64.gerchberg_saxton_f64(t, s, initial_phase=phi30)
        with _lib.Plan(_lib.ALGO_GS, 1, n, n, _lib.TGT_F32, False, s) as p:
            p.set_target(t[None])
            p.set_phase(phi30[None])
            p.run(s)
            ph, e, st, _ = p.read()
        de = np.abs(e[0] / e[0].max() - e_ref / e_ref.max()).max()
        print(f"{n} +{s}: phase rms {orc.phase_rms(ph[0], ref):.3e} |C|^2 max dev {de:.2e} "
              f"err rel {abs(st[0, s - 1, 3] / err_ref[-1] - 1):.2e}", flush=True)


if __name__ == "__main__":
    main()
