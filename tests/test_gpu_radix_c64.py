"""The complex64 radix-plan back end of the any-size engine
(csrc/radix_c128.hpp at P = PREC_F32, rz_inst.hip): GS with a float32 target
on image sides that the float32 engine has no plan for but that are 13-smooth
SLM panel lengths (plans.hpp variant 3: 600, 800, 1000, 1080, 1152, 1200,
1280, 1536, 1920), e.g. a 1080 x 1920 panel -- complex64 state and float32
butterflies like the float32 engine (kernels.hpp) on 2^k sides, on the
Stockham radix kernels instead of the float64 mixed radix.

The float32 engine's bar applies (warm start from the oracle's
30-iteration phase, phase rms <= 1e-5 against the faithful float64 oracle);
uint8 targets, GD, $SLM_ENGINE=float64 and slm_plan_set_precision(F64) run
the same plans at float64 (tests/test_gpu_radix_c128.py holds them to 1e-6).
"""
import os

import numpy as np
import pytest

from oracle import gs_gd_oracle as orc

PHASE_RMS_TOL = 1e-5
PANELS = [(1080, 1920), (1920, 1080), (1200, 1920), (600, 800), (1000, 1024), (768, 1280), (1152, 1536)]


@pytest.fixture
def c64_engine(monkeypatch):
    monkeypatch.delenv("SLM_ENGINE", raising=False)
    monkeypatch.delenv("SLM_GENERIC_ENGINE", raising=False)
    monkeypatch.delenv("SLM_PRECISION", raising=False)
    yield
    from spatial_light_modulator_module_amd import algorithms as alg

    alg.clear_plans()


def _target(shape, u8=False, seed=0):
    rng = np.random.default_rng(seed)
    if u8:
        return rng.integers(0, 256, shape).astype(np.uint8)
    return rng.uniform(0, 255, shape).astype(np.float32)


def _workers():
    import scipy.fft as sfft

    return sfft.set_workers(min(16, os.cpu_count() or 1))  # the GPU box's CPU share


@pytest.mark.gpu
@pytest.mark.parametrize("shape", PANELS)
def test_c64_engine_selection(gpu, c64_engine, monkeypatch, shape):
    """float32 GS on a panel shape runs the complex64 radix kernels; uint8,
    GD, $SLM_ENGINE=float64 and an explicit float64 precision run the same
    mixed plans at float64 (complex128 state); $SLM_GENERIC_ENGINE=mr the
    float64 mixed radix."""
    h, w = shape
    with gpu.Plan(gpu.ALGO_GS, 1, h, w, gpu.TGT_F32, False, 2) as p:
        assert p.engine() == ("radix-c64", "radix-c64") and p.info()["precision"] == "f32"
        p.set_precision(gpu.PRECISION_F64)
        assert p.engine() == ("radix-c128", "radix-c128") and p.info()["precision"] == "f64"
        p.set_precision(gpu.PRECISION_F32)
        assert p.engine() == ("radix-c64", "radix-c64")
    with gpu.Plan(gpu.ALGO_GS, 1, h, w, gpu.TGT_U8, False, 2) as p:
        assert p.engine() == ("radix-c128", "radix-c128") and p.info()["precision"] == "f64"
    with gpu.Plan(gpu.ALGO_GD, 1, h, w, gpu.TGT_F32, False, 2) as p:
        assert p.engine() == ("radix-c128", "radix-c128")
    monkeypatch.setenv("SLM_ENGINE", "float64")
    with gpu.Plan(gpu.ALGO_GS, 1, h, w, gpu.TGT_F32, False, 2) as p:
        assert p.engine() == ("radix-c128", "radix-c128")
    monkeypatch.setenv("SLM_GENERIC_ENGINE", "mr")
    with gpu.Plan(gpu.ALGO_GS, 1, h, w, gpu.TGT_F32, False, 2) as p:
        assert p.engine() == ("mixed-radix", "mixed-radix")


@pytest.mark.gpu
@pytest.mark.parametrize("shape", PANELS)
def test_c64_fft2_vs_numpy(gpu, c64_engine, shape):
    """slm_fft2 (complex64 in and out) on the complex64 radix kernels: float32
    transform accuracy against numpy's float64 transform."""
    rng = np.random.default_rng(1)
    x = (rng.standard_normal((2,) + shape) + 1j * rng.standard_normal((2,) + shape)).astype(np.complex64)
    for inverse in (False, True):
        got = gpu.fft2(x, inverse=inverse)
        xx = x.astype(np.complex128)
        want = np.fft.ifft2(xx) * (shape[0] * shape[1]) if inverse else np.fft.fft2(xx)
        err = np.sqrt(np.mean(np.abs(got - want) ** 2) / np.mean(np.abs(want) ** 2))
        print(f"[parity] radix-c64 fft2 {shape} {'inverse' if inverse else 'forward'}: rel rms {err:.2e}")
        assert err < 1e-6, (shape, inverse, err)  # float32 butterflies: ~1e-7 measured by the 2^k engine


@pytest.mark.gpu
@pytest.mark.parametrize("shape,iters", [((1080, 1920), 100), ((1920, 1080), 100), ((600, 800), 200),
                                         ((1000, 1024), 200), ((1152, 1536), 100)])
def test_c64_gs_warm_start_vs_oracle(gpu, c64_engine, shape, iters):
    """SURVEY.md 8c warm-start protocol against the faithful float64 oracle:
    the float32 engine's bar (1e-5 rms), error curve and expected output."""
    t = _target(shape, seed=shape[0] + 7)
    with _workers():
        phi30, _, _ = orc.gerchberg_saxton_faithful(t, 30)
        phi30 = phi30.astype(np.float32)
        ref, ref_e, ref_err = orc.gerchberg_saxton_faithful(t, iters, initial_phase=phi30)
    with gpu.Plan(gpu.ALGO_GS, 1, shape[0], shape[1], gpu.TGT_F32, False, iters) as p:
        assert p.engine() == ("radix-c64", "radix-c64")
        p.set_target(t[None])
        p.set_phase(phi30[None])
        p.run(iters)
        ph, e, stats, _ = p.read()
    rms = orc.phase_rms(ph[0], ref)
    print(f"[parity] radix-c64 GS {shape} float32 target, warm 30+{iters}: phase rms {rms:.3e}")
    assert rms < PHASE_RMS_TOL
    # float32 statistics of complex64 transforms: 2.0e-5 at 1080 x 1920 +100 (profiles/r06)
    np.testing.assert_allclose(stats[0, :iters, 3], ref_err, rtol=1e-4)
    expected = e[0].astype(np.float64) * (float(np.max(t)) / stats[0, iters - 1, 0])
    np.testing.assert_allclose(expected, ref_e, rtol=1e-3, atol=1e-4 * float(np.max(ref_e)))


@pytest.mark.gpu
def test_c64_matches_float64_engine(gpu, c64_engine):
    """The same warm-started batch on the complex64 radix kernels and on the
    float64 ones (slm_plan_set_precision): phases within the float32 bar of
    each other, error curves at float32 accuracy."""
    t = np.stack([_target((600, 800), seed=s) for s in (1, 2)])
    phi = np.random.default_rng(3).uniform(-np.pi, np.pi, t.shape).astype(np.float32)
    out = {}
    with gpu.Plan(gpu.ALGO_GS, 2, 600, 800, gpu.TGT_F32, False, 10) as p:
        p.set_target(t)
        for prec in (gpu.PRECISION_F32, gpu.PRECISION_F64):
            p.set_precision(prec)
            p.set_phase(phi)
            p.run(10)
            out[prec] = (p.engine(), p.read())
    (eng32, (ph32, _, st32, _)), (eng64, (ph64, _, st64, _)) = out[gpu.PRECISION_F32], out[gpu.PRECISION_F64]
    assert eng32[0] == "radix-c64" and eng64[0] == "radix-c128"
    for b in range(2):
        rms = orc.phase_rms(ph32[b], ph64[b])
        print(f"[parity] radix-c64 vs radix-c128 GS 600x800 hologram {b}, 10 iterations: phase rms {rms:.3e}")
        assert rms < PHASE_RMS_TOL
    np.testing.assert_allclose(st32[:, :10, 3], st64[:, :10, 3], rtol=1e-5)


@pytest.mark.gpu
def test_c64_tolerance_stop_and_intensity(gpu, c64_engine):
    """A checked batch stops each hologram where `while error > tolerance`
    ends (src/algorithms.py:29), and slm_fft2_intensity on a panel shape."""
    t = np.stack([_target((600, 800), seed=s) for s in (7, 8)])
    loops = 20
    with gpu.Plan(gpu.ALGO_GS, 2, 600, 800, gpu.TGT_F32, False, loops) as p:
        assert p.engine() == ("radix-c64", "radix-c64")
        p.set_target(t)
        p.set_phase(None)
        p.run(loops)
        _, _, full, _ = p.read()
        tol = float(np.sqrt(full[0, 7, 3] * full[0, 8, 3]))
        stop0 = int(np.argmax(~(full[0, :loops, 3] > tol)))
        p.set_phase(None)
        p.run(loops, tol, True)
        _, _, st, it = p.read()
    assert it[0] == stop0 + 1
    np.testing.assert_allclose(st[0, :stop0 + 1, 3], full[0, :stop0 + 1, 3], rtol=1e-12)
    rng = np.random.default_rng(4)
    ph = rng.uniform(-np.pi, np.pi, (2, 600, 800)).astype(np.float32)
    got = gpu.fft2_intensity(ph)
    want = np.abs(np.fft.fft2(np.exp(1j * ph.astype(np.float64)))) ** 2
    np.testing.assert_allclose(got, want, rtol=1e-3, atol=2e-5 * float(want.max()))


@pytest.mark.gpu
def test_c64_incoming_amplitude(gpu, c64_engine):
    """An incoming intensity (src/algorithms.py:14-19) on a panel shape,
    warm-started as SURVEY.md 8c, against the faithful float64 oracle."""
    from spatial_light_modulator_module_amd import algorithms as alg

    shape = (600, 800)
    rng = np.random.default_rng(12)
    ain = np.sqrt(rng.uniform(0.25, 2.0, shape)).astype(np.float32)
    inten = ain.astype(np.float64) ** 2
    t = _target(shape, seed=13)
    phi30, _, _ = orc.gerchberg_saxton_faithful(t, 30, incoming_intensity=inten)
    phi30 = phi30.astype(np.float32)
    ph, _, errs, _, _ = alg.run_gs(t[None], 60, ain=ain, initial_phase=phi30[None])
    ref, _, ref_err = orc.gerchberg_saxton_faithful(t, 60, incoming_intensity=inten, initial_phase=phi30)
    rms = orc.phase_rms(ph[0], ref)
    print(f"[parity] radix-c64 GS {shape} with a_in, warm 30+60: phase rms {rms:.3e}")
    assert rms < PHASE_RMS_TOL
    np.testing.assert_allclose(errs[0], ref_err, rtol=1e-5)
