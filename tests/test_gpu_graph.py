"""Graph-replayed runs (slm_plan_run captures the whole enqueue once and
replays it): a reused plan must give the same bits as a fresh plan after
every change the cached graph could miss -- a new loop count, new phase data
in the same buffers, a precision switch (new kernels and twiddle tables)."""
import numpy as np
import pytest


def _inputs(n=128, seed=7):
    rng = np.random.default_rng(seed)
    t = rng.uniform(0, 255, (1, n, n)).astype(np.float32)
    phi1 = rng.uniform(0, 2 * np.pi, (1, n, n)).astype(np.float32)
    phi2 = rng.uniform(0, 2 * np.pi, (1, n, n)).astype(np.float32)
    return t, phi1, phi2


def _fresh(lib, t, phi, loops, precision):
    with lib.Plan(lib.ALGO_GS, 1, t.shape[1], t.shape[2], lib.TGT_F32, False, 16) as p:
        p.set_precision(precision)
        p.set_target(t)
        p.set_phase(phi)
        p.run(loops)
        ph, _, stats, _ = p.read(expected=False)
    return ph, stats


@pytest.mark.gpu
def test_reused_plan_matches_fresh_plans(gpu):
    lib = gpu
    t, phi1, phi2 = _inputs()
    with lib.Plan(lib.ALGO_GS, 1, t.shape[1], t.shape[2], lib.TGT_F32, False, 16) as p:
        p.set_precision(lib.PRECISION_F32)
        p.set_target(t)
        steps = [(phi1, 5, lib.PRECISION_F32), (phi2, 5, lib.PRECISION_F32), (phi2, 9, lib.PRECISION_F32),
                 (phi1, 9, lib.PRECISION_F64), (phi1, 9, lib.PRECISION_F32)]
        for phi, loops, prec in steps:
            if p.precision != prec:
                p.set_precision(prec)
            p.set_phase(phi)
            p.run(loops)
            ph, _, stats, _ = p.read(expected=False)
            ref_ph, ref_stats = _fresh(lib, t, phi, loops, prec)
            np.testing.assert_array_equal(ph, ref_ph)
            np.testing.assert_array_equal(stats[:, :loops], ref_stats[:, :loops])
