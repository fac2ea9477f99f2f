import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import gs_gd_oracle as orc
from spatial_light_modulator_module_amd import _lib
from spatial_light_modulator_module_amd import algorithms as alg
_lib.init(0)
shape = (512, 2048)
rng = np.random.default_rng(shape[0] * 7 + shape[1])
t = rng.uniform(0, 255, shape).astype(np.float32)
phi0 = rng.uniform(-np.pi, np.pi, shape)
for plan in ("wide", "narrow"):
    os.environ["SLM_PLAN"] = plan
    for k in (1, 2, 3, 4, 6, 12):
        alg.clear_plans()
        ph, e, errs, norm, emax = alg.run_gs(t[None], k, initial_phase=phi0[None])
        pf, ef, errf = orc.gerchberg_saxton_faithful(t, k, initial_phase=phi0.astype(np.float32))
        d = np.abs(np.angle(np.exp(1j * (ph[0] - pf))))
        bad = np.argwhere(d > 1e-3)
        print(plan, k, f"rms {orc.phase_rms(ph[0], pf):.2e} err_rel {abs(errs[0][-1]/errf[-1]-1):.1e} nbad {len(bad)}",
              bad[:4].tolist(), flush=True)
