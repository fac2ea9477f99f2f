import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatial_light_modulator_module_amd import _lib
from spatial_light_modulator_module_amd import algorithms as alg
_lib.init(0)
def check(label, fn, reps=8):
    outs = [fn() for _ in range(reps)]
    diff = [int(not np.array_equal(outs[0], o)) for o in outs]
    print(label, "nondeterministic reps:", sum(diff), flush=True)
for shape in [(512, 2048), (64, 2048), (2048, 2048), (1024, 4096), (4096, 512)]:
    rng = np.random.default_rng(5)
    x = (rng.standard_normal(shape) + 1j * rng.standard_normal(shape)).astype(np.complex64)
    t = rng.uniform(0, 255, shape).astype(np.float32)
    phi0 = rng.uniform(-np.pi, np.pi, shape)
    for plan in ("wide", "narrow"):
        os.environ["SLM_PLAN"] = plan
        alg.clear_plans()
        check(f"{shape} {plan} fft2", lambda: _lib.fft2(x))
        check(f"{shape} {plan} ifft2", lambda: _lib.fft2(x, inverse=True))
        check(f"{shape} {plan} gs x3", lambda: alg.run_gs(t[None], 3, initial_phase=phi0[None])[0])
