"""The wave-shuffle transform pair (csrc/fft_shuffle.hpp) of the 1024-point GS
kernels: which plans run it, and its parity with the float64 restatement of
src/algorithms.py:10-49 (oracle/gs_gd_oracle.py, pinned to the reference
goldens by tests/test_oracle_golden.py).

The pair runs the first transform of each GS half-iteration decimated in
frequency and the second decimated in time, with four of its six exchanges as
v_permlane16/32 swaps (register <-> lane bit) and two through LDS; the
schedule is simulated lane by lane in tools/shuffle_fft_model.py (not a GPU
test: `test_shuffle_model` runs it on the CPU).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import gs_gd_oracle as orc

PHASE_RMS_TOL = 1e-5
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class env:
    def __init__(self, **kw):
        self.kw = kw

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kw}
        os.environ.update({k: str(v) for k, v in self.kw.items()})

    def __exit__(self, *exc):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_shuffle_model():
    """CPU: the lane-level model of the schedule matches numpy.fft and its LDS
    exchange is bank-conflict-free."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "shuffle_fft_model.py")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "model ok" in r.stdout
    for line in r.stdout.splitlines():
        if "extra cycles" in line or line.startswith("X2^H"):
            assert all(int(tok) == 0 for tok in line.replace(":", " ").split() if tok.isdigit()), line


@pytest.mark.gpu
def test_engine_selection(gpu):
    """GS and GD float32 plans and GS float64 plans with 1024-point narrow
    lines run the shuffle pair on that axis (float64: double values between
    its passes, r05); GD float64 and the wide batched plan keep the Stockham
    pair."""
    lib = gpu
    cases = [
        ((1, 1024, 1024), lib.ALGO_GS, lib.PRECISION_F32, ("shuffle", "shuffle")),
        ((2, 1024, 1024), lib.ALGO_GS, lib.PRECISION_F32, ("shuffle", "shuffle")),
        ((1, 768, 1024), lib.ALGO_GS, lib.PRECISION_F32, ("stockham", "shuffle")),
        ((1, 1024, 768), lib.ALGO_GS, lib.PRECISION_F32, ("shuffle", "stockham")),
        ((1, 1024, 1024), lib.ALGO_GS, lib.PRECISION_F64, ("shuffle", "shuffle")),
        ((1, 1024, 1024), lib.ALGO_GD, lib.PRECISION_F64, ("stockham", "stockham")),
        ((1, 1024, 1024), lib.ALGO_GD, lib.PRECISION_F32, ("shuffle", "shuffle")),
        ((64, 1024, 1024), lib.ALGO_GS, lib.PRECISION_F32, ("stockham", "stockham")),
    ]
    for (b, h, w), algo, prec, want in cases:
        with lib.Plan(algo, b, h, w, lib.TGT_F32, False, 4) as p:
            p.set_precision(prec)
            info = p.info()
        assert info["engine"] == want, (b, h, w, algo, prec, info)
    with env(SLM_PLAN="narrow"):
        with lib.Plan(lib.ALGO_GS, 64, 1024, 1024, lib.TGT_F32, False, 4) as p:
            assert p.info()["engine"] == ("shuffle", "shuffle")


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(1024, 1024), (768, 1024), (1024, 768)])
@pytest.mark.parametrize("dtype", [np.uint8, np.float32])
def test_shuffle_gs_vs_oracle(gpu, shape, dtype):
    """Random-phase warm start, 6 iterations (not chaotic over so few): phase
    within 1e-5 rms of the float64 restatement, error curve to 1e-5."""
    from spatial_light_modulator_module_amd import algorithms as alg

    rng = np.random.default_rng(shape[0] * 3 + shape[1] + (dtype == np.uint8))
    t = rng.integers(0, 256, shape).astype(dtype) if dtype == np.uint8 else rng.uniform(0, 255, shape).astype(
        dtype)
    phi0 = rng.uniform(-np.pi, np.pi, shape)
    loops = 6
    phase, e, errs, norm, emax = alg.run_gs(t[None], loops, initial_phase=phi0[None])
    ph_f, exp_f, err_f = orc.gerchberg_saxton_faithful(t, loops, initial_phase=phi0.astype(np.float32))
    rms = orc.phase_rms(phase[0], ph_f)
    print(f"[parity] shuffle GS {shape} {np.dtype(dtype).name} x{loops}: phase rms {rms:.3e}")
    assert rms < PHASE_RMS_TOL
    np.testing.assert_allclose(errs[0], err_f, rtol=1e-5)
    np.testing.assert_allclose(alg.expected_from(e[0], norm[0], emax[0]), exp_f, rtol=1e-3,
                               atol=1e-4 * float(norm[0]))


@pytest.mark.gpu
def test_shuffle_gs_incoming_intensity(gpu):
    """a_in (the reference's incoming intensity) is read by the row projection
    at the shuffle pair's element indices."""
    from spatial_light_modulator_module_amd import algorithms as alg

    n = 1024
    rng = np.random.default_rng(11)
    t = rng.uniform(0, 255, (n, n)).astype(np.float32)
    inten = rng.uniform(0.2, 1.0, (n, n))
    phi0 = rng.uniform(-np.pi, np.pi, (n, n))
    loops = 6
    ain = np.sqrt(inten).astype(np.float32)
    phase, e, errs, norm, emax = alg.run_gs(t[None], loops, ain=ain, initial_phase=phi0[None])
    ph_f, _, err_f = orc.gerchberg_saxton_faithful(t, loops, incoming_intensity=inten,
                                                    initial_phase=phi0.astype(np.float32))
    rms = orc.phase_rms(phase[0], ph_f)
    print(f"[parity] shuffle GS 1024^2 with incoming intensity x{loops}: phase rms {rms:.3e}")
    assert rms < PHASE_RMS_TOL
    np.testing.assert_allclose(errs[0], err_f, rtol=1e-5)


@pytest.mark.gpu
def test_shuffle_batch_equals_single(gpu):
    """Holograms of a batch on the shuffle pair (forced narrow plan for 4
    images) equal single runs bit for bit."""
    lib = gpu
    n, loops = 1024, 12
    rng = np.random.default_rng(5)
    t = rng.uniform(0, 255, (4, n, n)).astype(np.float32)
    phi = rng.uniform(-np.pi, np.pi, t.shape).astype(np.float32)

    def run(tt, ph):
        with lib.Plan(lib.ALGO_GS, tt.shape[0], n, n, lib.TGT_F32, False, loops) as p:
            assert p.info()["engine"] == ("shuffle", "shuffle")
            p.set_target(tt)
            p.set_phase(ph)
            p.run(loops)
            return p.read()[:3]

    with env(SLM_PLAN="narrow"):
        batch = run(t, phi)
        for k in (0, 3):
            one = run(t[k:k + 1], phi[k:k + 1])
            for a, b in zip(batch, one):
                np.testing.assert_array_equal(a[k], b[0])
