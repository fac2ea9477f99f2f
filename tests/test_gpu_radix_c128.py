"""The complex128 radix-plan back end of the any-size engine
(csrc/radix_c128.hpp, rz_inst.hip): image sides with a radix plan (2^k, 768)
under $SLM_ENGINE=float64 -- complex128 state, float64 butterflies and
complex128 LDS exchanges, the reference's own dtypes (src/algorithms.py:27-38,
83-93) at radix-plan speed.

Held to the faithful float64 oracle (oracle/gs_gd_oracle.py, pinned to the
reference goldens in test_oracle_golden.py) at the float32 phase output's
rounding, and to the mixed-radix back end (same contract, other transform
rounding) far inside that. The configs' own run lengths (4096^2 at 200
iterations, GD 1024^2 at 500) are gated in test_gpu_configs.py.
"""
import numpy as np
import pytest

from oracle import gs_gd_oracle as orc


@pytest.fixture
def f64_engine(monkeypatch):
    """Plans of the test are created on the complex128 engine ($SLM_ENGINE=float64)."""
    monkeypatch.setenv("SLM_ENGINE", "float64")
    monkeypatch.delenv("SLM_GENERIC_ENGINE", raising=False)
    yield
    from spatial_light_modulator_module_amd import algorithms as alg

    alg.clear_plans()


def _target(shape, u8, seed=0):
    rng = np.random.default_rng(seed)
    if u8:
        return rng.integers(0, 256, shape).astype(np.uint8)
    return rng.uniform(0, 255, shape).astype(np.float32)


def _gs(lib, t, loops, phase=None, tol=0.0, checked=False, want="radix-c128"):
    b, h, w = t.shape
    with lib.Plan(lib.ALGO_GS, b, h, w, lib.TGT_U8 if t.dtype == np.uint8 else lib.TGT_F32, False, loops) as p:
        assert p.engine() == (want, want) and p.info()["precision"] == "f64", p.engine()
        p.set_target(t)
        p.set_phase(phase)
        p.run(loops, tol, checked)
        return p.read()


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(64, 64), (128, 256), (768, 1024), (1024, 1024), (256, 2048), (4096, 512),
                                   (1080, 1920), (1920, 1080), (600, 800), (1200, 1280), (1000, 1536), (1152, 1152)])
def test_rz_fft2_c128_vs_numpy(gpu, f64_engine, shape):
    """slm_fft2_c128 on the radix-plan kernels (every plan key the engine
    picks at these shapes) against numpy.fft at float64 accuracy."""
    rng = np.random.default_rng(2)
    x = rng.standard_normal((2,) + shape) + 1j * rng.standard_normal((2,) + shape)
    for inverse in (False, True):
        got = gpu.fft2_c128(x, inverse=inverse)
        want = np.fft.ifft2(x) * (shape[0] * shape[1]) if inverse else np.fft.fft2(x)
        err = np.max(np.abs(got - want)) / np.max(np.abs(want))
        assert err < 1e-13, (shape, inverse, err)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(128, 256), (768, 1024), (1024, 1024), (600, 800), (1080, 1920)])
@pytest.mark.parametrize("u8", [False, True])
def test_rz_gs_warm_start_vs_oracle(gpu, f64_engine, shape, u8):
    """SURVEY.md 8c warm-start protocol (the oracle's phase after 30 cold
    iterations, then 60 more) against the faithful float64 oracle."""
    t = _target(shape, u8, seed=shape[0])
    phi30, _, _ = orc.gerchberg_saxton_faithful(t, 30)
    phi30 = phi30.astype(np.float32)
    ref, ref_e, ref_err = orc.gerchberg_saxton_faithful(t, 60, initial_phase=phi30)
    ph, e, stats, iters = _gs(gpu, t[None], 60, phi30[None])
    rms = orc.phase_rms(ph[0], ref)
    print(f"[parity] radix-c128 GS {shape} {'u8' if u8 else 'f32'} warm 30+60: phase rms {rms:.3e}")
    assert rms < 1e-6  # float32 phase output: its rounding is ~1e-7
    np.testing.assert_allclose(stats[0, :, 3], ref_err, rtol=1e-6)
    expected = e[0].astype(np.float64) * (float(np.max(t)) / stats[0, -1, 0])
    np.testing.assert_allclose(expected, ref_e, rtol=1e-6, atol=1e-6 * float(np.max(ref_e)))
    assert (iters == -1).all()


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["rm", "b2"])
def test_rz_matches_mixed_radix(gpu, monkeypatch, layout):
    """Both complex128 back ends on one warm-started batch, the radix kernels on
    each state layout (radix_c128.hpp LAY_RM / LAY_B2): the same contract,
    transforms that round differently (~1e-16), so phases and error curves
    agree far inside the float32 output's rounding."""
    monkeypatch.setenv("SLM_ENGINE", "float64")
    monkeypatch.setenv("SLM_RZ_LAYOUT", layout)
    t = np.stack([_target((256, 512), False, seed=s) for s in (1, 2)])
    phi = np.random.default_rng(3).uniform(-np.pi, np.pi, t.shape).astype(np.float32)
    monkeypatch.delenv("SLM_GENERIC_ENGINE", raising=False)
    ph_z, e_z, st_z, _ = _gs(gpu, t, 25, phi)
    monkeypatch.setenv("SLM_GENERIC_ENGINE", "mr")
    ph_m, e_m, st_m, _ = _gs(gpu, t, 25, phi, want="mixed-radix")
    d = float(np.max(np.abs(np.angle(np.exp(1j * (ph_z.astype(np.float64) - ph_m))))))
    print(f"[parity] radix-c128 ({layout}) vs mixed-radix GS 2 x 256x512, 25 iterations: max phase difference {d:.3e}")
    assert d < 1e-5  # float32 outputs: an angle near a rounding boundary moves by one float32 ulp
    np.testing.assert_allclose(st_z[:, :25, 3], st_m[:, :25, 3], rtol=1e-10)
    np.testing.assert_allclose(e_z, e_m, rtol=1e-6)


def _gd_run(lib, t, loops, x0):
    shape = t.shape
    with lib.Plan(lib.ALGO_GD, 1, shape[0], shape[1], lib.TGT_F32, False, loops) as p:
        eng = p.engine()
        p.set_target(t[None])
        if x0 is not None:
            p.set_field(x0[None])
        p.set_lr(np.full(loops, 0.005, np.float32))
        p.run(loops, white_attention=1.0)
        ph, _, stats, _ = p.read()
    return eng, ph[0], stats[0, :loops, 3]


@pytest.mark.gpu
@pytest.mark.parametrize("engine", ["radix-c128", "radix-c128-rm", "mixed-radix"])
def test_rz_gd_vs_oracle(gpu, monkeypatch, engine):
    """GD (src/algorithms.py:60-112) on both complex128 back ends (the radix
    kernels on their default B2 layout and on the row-major one) from the
    random guess (set on the host, seed 42), against the faithful float64 oracle."""
    monkeypatch.setenv("SLM_ENGINE", "float64")
    if engine == "radix-c128-rm":
        monkeypatch.setenv("SLM_RZ_LAYOUT", "rm")
        engine = "radix-c128"
    if engine == "mixed-radix":
        monkeypatch.setenv("SLM_GENERIC_ENGINE", "mr")
    else:
        monkeypatch.delenv("SLM_GENERIC_ENGINE", raising=False)
    from spatial_light_modulator_module_amd import algorithms as alg

    shape = (128, 256) if engine == "radix-c128" else (96, 160)
    t = _target(shape, False, seed=5)
    loops = 40
    x0 = alg.make_initial_guess("random", None, t, 42)
    ref, _, ref_err, _ = orc.gradient_descent_faithful(t, loops, 0.005, 1.0, 0, initial_field=x0)
    eng, ph, err = _gd_run(gpu, t, loops, x0)
    assert eng == (engine, engine), eng
    rms = orc.phase_rms(ph, ref)
    print(f"[parity] {engine} GD {shape} random guess, {loops} iterations: phase rms {rms:.3e}")
    # the field crosses the C-ABI as complex64 (3.3e-6 after 60 iterations at 96 x 160, CPU check)
    assert rms < 1e-5
    np.testing.assert_allclose(err, ref_err, rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("engine", ["radix-c128", "mixed-radix"])
def test_gd_fourier_guess_on_the_complex128_engines(gpu, monkeypatch, engine):
    """GD from the "fourier" guess a_in exp(i angle(ifft2(sqrt T))) formed on
    the device (src/algorithms.py:153-156; the field is never set, so each
    engine's CO_AMP_INV + RO_GD_FOURIER path runs -- on the mixed-radix engine
    the field is then kept in digit-reversed row order). That start is
    Hermitian-symmetric, so the run is chaotic at rounding level like GS's
    cold start: after one iteration the phase is gated pointwise
    (the guess itself), the first errors pointwise, the last in a band."""
    monkeypatch.setenv("SLM_ENGINE", "float64")
    if engine == "mixed-radix":
        monkeypatch.setenv("SLM_GENERIC_ENGINE", "mr")
    else:
        monkeypatch.delenv("SLM_GENERIC_ENGINE", raising=False)
    shape = (128, 256) if engine == "radix-c128" else (96, 160)
    t = _target(shape, False, seed=5)
    ref1, _, _, _ = orc.gradient_descent_faithful(t, 1, 0.005, 1.0, 0, initial_guess="fourier")
    eng, ph1, _ = _gd_run(gpu, t, 1, None)
    assert eng == (engine, engine), eng
    rms1 = orc.phase_rms(ph1, ref1)
    loops = 40
    ref, _, ref_err, _ = orc.gradient_descent_faithful(t, loops, 0.005, 1.0, 0, initial_guess="fourier")
    _, ph, err = _gd_run(gpu, t, loops, None)
    print(f"[parity] {engine} GD {shape} fourier guess: phase rms {rms1:.3e} after 1 iteration; "
          f"final error {err[-1]:.4e} (oracle {ref_err[-1]:.4e})")
    assert rms1 < 1e-6
    np.testing.assert_allclose(err[:3], ref_err[:3], rtol=1e-6)
    assert 0.5 < err[-1] / ref_err[-1] < 2.0


@pytest.mark.gpu
def test_rz_tolerance_stop(gpu, f64_engine):
    """A checked run stops each hologram where `while error > tolerance` ends
    (src/algorithms.py:29): the stopped hologram equals an unchecked run of
    that many iterations; the other keeps going."""
    t = np.stack([_target((128, 128), False, seed=s) for s in (7, 8)])
    loops = 20
    _, _, full, _ = _gs(gpu, t, loops)
    tol = float(np.sqrt(full[0, 7, 3] * full[0, 8, 3]))
    stop0 = int(np.argmax(~(full[0, :loops, 3] > tol)))
    ph, e, st, it = _gs(gpu, t, loops, tol=tol, checked=True)
    assert it[0] == stop0 + 1
    ph0, e0, st0, _ = _gs(gpu, t[:1], stop0 + 1)
    np.testing.assert_array_equal(ph[0], ph0[0])
    np.testing.assert_allclose(st[0, :stop0 + 1], st0[0, :stop0 + 1], rtol=1e-12)
    np.testing.assert_array_equal(e[0], e0[0])


@pytest.mark.gpu
def test_rz_incoming_amplitude(gpu, f64_engine):
    """An incoming intensity (src/algorithms.py:14-19 / :65-70) on the radix
    back end: GS (uint8 target, warm start) and GD (random guess scaled by a_in)."""
    from spatial_light_modulator_module_amd import algorithms as alg

    shape = (128, 256)
    rng = np.random.default_rng(12)
    ain = np.sqrt(rng.uniform(0.25, 2.0, shape)).astype(np.float32)
    inten = ain.astype(np.float64) ** 2
    t = _target(shape, True, seed=13)
    phi30, _, _ = orc.gerchberg_saxton_faithful(t, 30, incoming_intensity=inten)
    phi30 = phi30.astype(np.float32)
    ph, _, errs, _, _ = alg.run_gs(t[None], 30, ain=ain, initial_phase=phi30[None])
    ref, _, ref_err = orc.gerchberg_saxton_faithful(t, 30, incoming_intensity=inten, initial_phase=phi30)
    rms = orc.phase_rms(ph[0], ref)
    print(f"[parity] radix-c128 GS {shape} uint8 with a_in, warm 30+30: phase rms {rms:.3e}")
    assert rms < 1e-6
    np.testing.assert_allclose(errs[0], ref_err, rtol=1e-6)
    tf = _target(shape, False, seed=14)
    x0 = alg.make_initial_guess("random", inten ** 0.5, tf, 42)
    ph, _, errs, _, _ = alg.run_gd(tf[None], 40, np.full(40, 0.005), 1.0, ain=ain, initial_field=x0[None])
    ref, _, ref_err, _ = orc.gradient_descent_faithful(tf, 40, 0.005, 1.0, 0, incoming_intensity=inten,
                                                       initial_field=x0)
    assert orc.phase_rms(ph[0], ref) < 1e-5
    np.testing.assert_allclose(errs[0], ref_err, rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("guess", ["random", "fourier"])
def test_rz_gd_panel_vs_oracle(gpu, monkeypatch, guess):
    """GD on a 13-smooth SLM panel (600 x 800: mixed plans 10.6.10 / 10.8.10 at
    float64, the default GD engine there) against the faithful float64 oracle,
    from the host-set random guess and from the device-formed "fourier" guess
    (chaotic like GS's cold start: first errors pointwise, the last in a band)."""
    monkeypatch.delenv("SLM_ENGINE", raising=False)
    monkeypatch.delenv("SLM_GENERIC_ENGINE", raising=False)
    from spatial_light_modulator_module_amd import algorithms as alg

    shape = (600, 800)
    t = _target(shape, False, seed=9)
    loops = 20
    x0 = alg.make_initial_guess("random", None, t, 42) if guess == "random" else None
    kw = {"initial_field": x0} if guess == "random" else {"initial_guess": "fourier"}
    ref, _, ref_err, _ = orc.gradient_descent_faithful(t, loops, 0.005, 1.0, 0, **kw)
    eng, ph, err = _gd_run(gpu, t, loops, x0)
    assert eng == ("radix-c128", "radix-c128"), eng
    rms = orc.phase_rms(ph, ref)
    print(f"[parity] radix-c128 GD {shape} {guess} guess, {loops} iterations: phase rms {rms:.3e}; "
          f"final error {err[-1]:.6e} (oracle {ref_err[-1]:.6e})")
    if guess == "random":
        assert rms < 1e-5  # the field crosses the C-ABI as complex64
        np.testing.assert_allclose(err, ref_err, rtol=1e-5)
    else:
        np.testing.assert_allclose(err[:3], ref_err[:3], rtol=1e-6)
        assert 0.5 < err[-1] / ref_err[-1] < 2.0
