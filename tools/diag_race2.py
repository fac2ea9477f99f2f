import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatial_light_modulator_module_amd import _lib
from spatial_light_modulator_module_amd import algorithms as alg
_lib.init(0)
shape = (512, 2048)
rng = np.random.default_rng(shape[0] * 7 + shape[1])
t = rng.uniform(0, 255, shape).astype(np.float32)
phi0 = rng.uniform(-np.pi, np.pi, shape)
ref = {}
for k in (12, 6, 3, 1):
    ref[k] = alg.run_gs(t[None], k, initial_phase=phi0[None])[0][0].copy()
bad = 0
for rep in range(40):
    if rep % 10 == 0:
        alg.clear_plans()
    ph = alg.run_gs(t[None], 12, initial_phase=phi0[None])[0][0]
    if not np.array_equal(ph, ref[12]):
        bad += 1
        d = np.argwhere(ph != ref[12])
        print("rep", rep, "differs at", len(d), "pixels; rows", np.unique(d[:, 0])[:10].tolist(),
              "cols", np.unique(d[:, 1])[:10].tolist(), flush=True)
        # find first iteration where it differs
        for k in (1, 3, 6):
            for _ in range(5):
                pk = alg.run_gs(t[None], k, initial_phase=phi0[None])[0][0]
                if not np.array_equal(pk, ref[k]):
                    dk = np.argwhere(pk != ref[k])
                    print("   k", k, "differs at", len(dk), "rows", np.unique(dk[:, 0])[:8].tolist(),
                          "cols", np.unique(dk[:, 1])[:8].tolist(), flush=True)
print("bad", bad, "of 40", flush=True)
