import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import gs_gd_oracle as orc
from spatial_light_modulator_module_amd import _lib
from spatial_light_modulator_module_amd import algorithms as alg
_lib.init(0)
for shape in [(512, 2048), (64, 2048), (2048, 64), (2048, 2048), (512, 512), (256, 2048)]:
    rng = np.random.default_rng(1)
    t = rng.uniform(0, 255, shape).astype(np.float32)
    phi0 = rng.uniform(-np.pi, np.pi, shape)
    x = (rng.standard_normal(shape) + 1j * rng.standard_normal(shape)).astype(np.complex64)
    for plan in ("wide", "narrow"):
        os.environ["SLM_PLAN"] = plan
        alg.clear_plans()
        ph, e, errs, norm, emax = alg.run_gs(t[None], 1, initial_phase=phi0[None])
        pf, _, _ = orc.gerchberg_saxton_faithful(t, 1, initial_phase=phi0.astype(np.float32))
        f = _lib.fft2(x); fi = _lib.fft2(x, inverse=True)
        ef = np.linalg.norm(f - np.fft.fft2(x)) / np.linalg.norm(f)
        efi = np.linalg.norm(fi - np.fft.ifft2(x) * x.size) / np.linalg.norm(fi)
        with alg.get_plan(_lib.ALGO_GS, 1, shape[0], shape[1], _lib.TGT_F32, False, 1) as p:
            info = p.info()
        print(shape, plan, "gs1 rms", f"{orc.phase_rms(ph[0], pf):.2e}", "fft", f"{ef:.1e}", "ifft", f"{efi:.1e}",
              info["row_plan"], info["col_plan"], info["row_threads"], info["col_threads"], flush=True)
