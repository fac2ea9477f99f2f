import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import gs_gd_oracle as orc
from spatial_light_modulator_module_amd import _lib
from spatial_light_modulator_module_amd import algorithms as alg
_lib.init(0)
shape = (512, 512)
rng = np.random.default_rng(1)
t = rng.uniform(0, 255, shape).astype(np.float32)
phi0 = rng.uniform(-np.pi, np.pi, shape)
pf, _, _ = orc.gerchberg_saxton_faithful(t, 1, initial_phase=phi0.astype(np.float32))
x = (rng.standard_normal(shape) + 1j * rng.standard_normal(shape)).astype(np.complex64)
for plan in ("wide", "narrow"):
    os.environ["SLM_PLAN"] = plan
    for prec in (_lib.PRECISION_F64, _lib.PRECISION_F32):
        alg.clear_plans()
        p = alg.get_plan(_lib.ALGO_GS, 1, 512, 512, _lib.TGT_F32, False, 1)
        p.set_precision(prec)
        ph, e, errs, norm, emax = alg.run_gs(t[None], 1, initial_phase=phi0[None])
        d = np.abs(np.angle(np.exp(1j * (ph[0] - pf))))
        rowm = d.max(axis=1); colm = d.max(axis=0)
        print(plan, "f64" if prec else "f32", f"rms {np.sqrt(np.mean(d*d)):.2e} p50 {np.median(d):.1e} p99 {np.percentile(d,99):.1e} max {d.max():.1e}",
              "worst rows", np.argsort(rowm)[-5:].tolist(), "worst cols", np.argsort(colm)[-5:].tolist(), flush=True)
        print("   col-max by x%4:", [f"{d[:, k::4].mean():.2e}" for k in range(4)], " row-mean by y%4:", [f"{d[k::4].mean():.2e}" for k in range(4)])
