#!/usr/bin/env python3
"""Phase distance between the GPU, the complex64 model and the float64
restatement along a warm-started GS trajectory (golden g1/g2)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import gs_gd_oracle as orc  # noqa: E402
from spatial_light_modulator_module_amd import _lib  # noqa: E402
from spatial_light_modulator_module_amd import algorithms as alg  # noqa: E402

_lib.init(0)
for name in ("g1_gs_u8_256.npz", "g2_gs_f32_256.npz"):
    g = np.load(os.path.join(ROOT, "tests", "golden", name))
    t, phi = g["target"], g["phi30"]
    for k in (1, 2, 5, 20, 50, 100, 200):
        pg, _, _, _, _ = alg.run_gs(t[None], k, initial_phase=phi[None])
        pm, _, _ = orc.gerchberg_saxton_c64(t, k, initial_phase=phi)
        pf, _, _ = orc.gerchberg_saxton_faithful(t, k, initial_phase=phi)
        print(f"{name} k={k:3d} gpu-f64 {orc.phase_rms(pg[0], pf):.3e} model-f64 {orc.phase_rms(pm, pf):.3e} "
              f"gpu-model {orc.phase_rms(pg[0], pm):.3e}", flush=True)
