import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import gs_gd_oracle as orc
from spatial_light_modulator_module_amd import _lib
from spatial_light_modulator_module_amd import algorithms as alg
_lib.init(0)
for shape in [(512, 2048), (256, 256), (768, 1024)]:
    rng = np.random.default_rng(shape[0] * 7 + shape[1])
    t = rng.uniform(0, 255, shape).astype(np.float32)
    phi0 = rng.uniform(-np.pi, np.pi, shape)
    pf, _, _ = orc.gerchberg_saxton_faithful(t, 12, initial_phase=phi0.astype(np.float32))
    outs = []
    for rep in range(6):
        if rep % 2 == 0:
            alg.clear_plans()
        ph, e, errs, norm, emax = alg.run_gs(t[None], 12, initial_phase=phi0[None])
        outs.append(ph[0].copy())
        print(shape, rep, f"rms {orc.phase_rms(ph[0], pf):.3e}", "identical to rep0:", bool(np.array_equal(outs[0], ph[0])), flush=True)
