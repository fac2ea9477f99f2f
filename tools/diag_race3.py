import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatial_light_modulator_module_amd import _lib
from spatial_light_modulator_module_amd import algorithms as alg
_lib.init(0)
reps = int(os.environ.get("REPS", "16"))
for shape in [(512, 2048), (2048, 512), (256, 2048), (512, 1024), (1024, 1024), (2048, 2048), (512, 512), (768, 1024)]:
    rng = np.random.default_rng(shape[0] * 7 + shape[1])
    t = rng.uniform(0, 255, shape).astype(np.float32)
    phi0 = rng.uniform(-np.pi, np.pi, shape)
    for plan in ("wide", "narrow"):
        os.environ["SLM_PLAN"] = plan
        alg.clear_plans()
        ref = alg.run_gs(t[None], 12, initial_phase=phi0[None])[0][0].copy()
        bad = sum(not np.array_equal(alg.run_gs(t[None], 12, initial_phase=phi0[None])[0][0], ref) for _ in range(reps))
        with alg.get_plan(_lib.ALGO_GS, 1, shape[0], shape[1], _lib.TGT_F32, False, 12) as p:
            inf = p.info()
        print(shape, plan, "row/col plan", inf["row_plan"], inf["col_plan"], "threads", inf["row_threads"], inf["col_threads"],
              "bad", bad, "of", reps, flush=True)
