"""Image shapes without a float32 radix plan: the any-size engine
(csrc/generic.hip) on both of its transform back ends for such sides.

The reference takes any (h, w) (src/algorithms.py:20-27; scipy.fft handles
every length). Sides outside SUPPORTED_LENGTHS run in complex128 state with
float64 arithmetic: on the hand-written mixed-radix kernels
(csrc/mixed_radix.hpp, mr_inst.hip) where both sides factor into 2..13, else
as 1-D line transforms along rows and transposed columns -- direct for a
mixed-radix side, Bluestein's chirp-z over a mixed-radix length for a side
with a larger prime factor (mr_line_kernel). Every test here runs on each
back end (`engine` fixture; $SLM_GENERIC_ENGINE=bluestein forces the line
transforms with chirp-z on every side), and both are held to the faithful
float64 oracle
(oracle/gs_gd_oracle.py, pinned to the reference goldens in
test_oracle_golden.py) far inside the north-star bar: warm-start GS and GD
phases at the float32 output's rounding (<= 1e-6 rms gated; the float32 FFT
path's bar is 1e-5), error curves at rtol 1e-6 (complex64 rounding of the warm
start's exp(1j phi) aside, 3e-8 measured).
"""
import argparse

import numpy as np
import pytest

from oracle import gs_gd_oracle as orc

SHAPES = [(96, 160), (45, 77), (768, 1000)]


def _smooth(n):
    for p in (2, 3, 5, 7, 11, 13):
        while n % p == 0:
            n //= p
    return n == 1


def _expected_engine(shape, engine):
    if engine == "mixed-radix" and all(_smooth(n) and n <= 8192 for n in shape):
        return "mixed-radix"
    return "bluestein"


@pytest.fixture(params=["mixed-radix", "bluestein"])
def engine(request, monkeypatch):
    """The back end the plans of one test are created on (read at plan creation)."""
    # "mr" keeps float32-target GS on shapes whose sides all have radix plans
    # (768 x 1000: complex64 radix kernels by default, test_gpu_radix_c64.py)
    # on the float64 mixed radix this file checks
    monkeypatch.setenv("SLM_GENERIC_ENGINE", "bluestein" if request.param == "bluestein" else "mr")
    yield request.param
    from spatial_light_modulator_module_amd import algorithms as alg

    alg.clear_plans()  # cached drop-in plans keep the engine they were created on


def _target(shape, u8, seed=0):
    rng = np.random.default_rng(seed)
    if u8:
        return rng.integers(0, 256, shape).astype(np.uint8)
    return rng.uniform(0, 255, shape).astype(np.float32)


def _gs(lib, t, loops, phase=None, tol=0.0, checked=False, engine="mixed-radix"):
    b, h, w = t.shape
    with lib.Plan(lib.ALGO_GS, b, h, w, lib.TGT_U8 if t.dtype == np.uint8 else lib.TGT_F32, False, loops) as p:
        want = _expected_engine((h, w), engine)
        assert p.engine() == (want, want) and p.info()["precision"] == "f64"
        p.set_target(t)
        p.set_phase(phase)
        p.run(loops, tol, checked)
        return p.read()


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(7, 33), (100, 60), (768, 1000), (1000, 1024), (97, 101), (1, 13), (2053, 2)])
def test_generic_fft2_vs_numpy(gpu, engine, shape):
    rng = np.random.default_rng(1)
    x = (rng.standard_normal((2,) + shape) + 1j * rng.standard_normal((2,) + shape)).astype(np.complex64)
    for inverse in (False, True):
        got = gpu.fft2(x, inverse=inverse)
        want = np.fft.ifft2(x.astype(np.complex128)) * (shape[0] * shape[1]) if inverse else np.fft.fft2(
            x.astype(np.complex128))
        err = np.max(np.abs(got - want)) / np.max(np.abs(want))
        assert err < 1e-6, err  # complex64 output rounding; the transforms are float64


@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("u8", [False, True])
def test_generic_gs_warm_start_vs_oracle(gpu, engine, shape, u8):
    """SURVEY.md 8c warm-start protocol (the reference's phase after 30
    cold iterations, then 60 more) against the faithful float64 oracle."""
    t = _target(shape, u8)
    phi30, _, _ = orc.gerchberg_saxton_faithful(t, 30)
    phi30 = phi30.astype(np.float32)
    ref, ref_e, ref_err = orc.gerchberg_saxton_faithful(t, 60, initial_phase=phi30)
    ph, e, stats, iters = _gs(gpu, t[None], 60, phi30[None], engine=engine)
    rms = orc.phase_rms(ph[0], ref)
    print(f"[parity] {engine} GS {shape} {'u8' if u8 else 'f32'} warm 30+60: phase rms {rms:.3e}")
    assert rms < 1e-6  # float32 phase output: its rounding is ~1e-7
    np.testing.assert_allclose(stats[0, :, 3], ref_err, rtol=1e-6)
    expected = e[0].astype(np.float64) * (float(np.max(t)) / stats[0, -1, 0])
    np.testing.assert_allclose(expected, ref_e, rtol=1e-6, atol=1e-6 * float(np.max(ref_e)))
    assert (iters == -1).all()


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(96, 160), (120, 90)])
def test_generic_gs_cold_start(gpu, engine, shape):
    """The cold start ifft2(sqrt T) in complex64 as the reference; the run is
    chaotic at rounding level after a few iterations, so the
    first errors are compared pointwise, the last in a band."""
    t = _target(shape, True, seed=3)
    ref, _, ref_err = orc.gerchberg_saxton_faithful(t, 40)
    ph, _, stats, _ = _gs(gpu, t[None], 40, engine=engine)
    np.testing.assert_allclose(stats[0, :3, 3], ref_err[:3], rtol=1e-6)
    # two float64 FFT libraries already end 1.4 rad apart after 50 cold iterations
    # (SURVEY.md 7): the final error is a band (1062 against 784 measured at 120 x 90)
    assert stats[0, -1, 3] < 0.5 * stats[0, 0, 3] and 0.5 < stats[0, -1, 3] / ref_err[-1] < 2.0


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(96, 160), (33, 50)])
def test_generic_gd_vs_oracle(gpu, engine, shape):
    from spatial_light_modulator_module_amd import algorithms as alg

    t = _target(shape, False, seed=5)
    loops = 60
    x0 = alg.make_initial_guess("random", None, t, 42)
    ref, ref_out, ref_err, _ = orc.gradient_descent_faithful(t, loops, 0.005, 1.0, 0, initial_field=x0)
    with gpu.Plan(gpu.ALGO_GD, 1, shape[0], shape[1], gpu.TGT_F32, False, loops) as p:
        want = _expected_engine(shape, engine)
        assert p.engine() == (want, want)
        p.set_target(t[None])
        p.set_field(x0[None])
        np.testing.assert_array_equal(p.read_field()[0], x0.astype(np.complex64))
        p.set_lr(np.full(loops, 0.005, np.float32))
        p.run(loops, white_attention=1.0)
        ph, e, stats, _ = p.read()
        x = p.read_field()[0]
    rms = orc.phase_rms(ph[0], ref)
    print(f"[parity] {engine} GD {shape} {loops} iterations: phase rms {rms:.3e}")
    # the initial field crosses the C-ABI as complex64: that rounding alone moves the
    # float64 oracle's phase by 3.3e-6 rms after 60 iterations at 96 x 160 (CPU check)
    assert rms < 1e-5
    np.testing.assert_allclose(stats[0, :loops, 3], ref_err, rtol=1e-5)  # 1.1e-6 measured
    assert np.isfinite(x).all()


@pytest.mark.gpu
def test_generic_tolerance_stop(gpu, engine):
    """A checked run stops each hologram where `while error > tolerance` ends
    (src/algorithms.py:29): the stopped hologram's phase, expected output and
    errors equal an unchecked run of that many iterations; the other keeps going."""
    t = np.stack([_target((64, 100), False, seed=s) for s in (7, 8)])
    loops = 20
    _, _, full, _ = _gs(gpu, t, loops, engine=engine)
    tol = float(np.sqrt(full[0, 7, 3] * full[0, 8, 3]))  # hologram 0 stops after iteration 9
    stop0 = int(np.argmax(~(full[0, :loops, 3] > tol)))
    ph, e, st, it = _gs(gpu, t, loops, tol=tol, checked=True, engine=engine)
    assert it[0] == stop0 + 1
    ph0, e0, st0, _ = _gs(gpu, t[:1], stop0 + 1, engine=engine)
    np.testing.assert_allclose(ph[0], ph0[0], atol=1e-6)
    np.testing.assert_allclose(st[0, :stop0 + 1], st0[0, :stop0 + 1], rtol=1e-10)
    np.testing.assert_allclose(e[0], e0[0], rtol=1e-6)
    ref, _, ref_err = orc.gerchberg_saxton_faithful(t[0], loops, tolerance=tol)
    assert len(ref_err) == stop0 + 1


@pytest.mark.gpu
def test_generic_drop_in_entry_points(gpu, engine):
    """gerchberg_saxton / gradient_descent (src/algorithms.py:10, :60) on a
    shape the CLI's resize would never produce: same triple as the reference."""
    from spatial_light_modulator_module_amd.algorithms import gerchberg_saxton, gradient_descent

    args = argparse.Namespace(incomming_intensity="uniform", tolerance=0.0, max_loops=15, gif=False,
                              print_info=False, plot_error=False, learning_rate=0.005, white_attention=1.0,
                              unsettle=0, initial_guess="random", random_seed=42)
    t = _target((50, 70), True, seed=9)
    holo, out, err = gerchberg_saxton(t, args)
    assert holo.dtype == np.float64 and holo.shape == t.shape and len(err) == 15
    _, _, ref_err = orc.gerchberg_saxton_faithful(t, 15)
    np.testing.assert_allclose(err[:3], ref_err[:3], rtol=1e-6)
    holo, out, err = gradient_descent(t.astype(np.float32), args)
    ref, ref_out, ref_err, _ = orc.gradient_descent_faithful(t.astype(np.float32), 15, 0.005, 1.0, 0)
    assert orc.phase_rms(holo, ref) < 1e-6
    np.testing.assert_allclose(err, ref_err, rtol=1e-6)


@pytest.mark.gpu
def test_generic_intensity_vs_numpy(gpu, engine):
    rng = np.random.default_rng(4)
    ph = rng.uniform(-np.pi, np.pi, (2, 48, 80)).astype(np.float32)
    got = gpu.fft2_intensity(ph)
    want = np.abs(np.fft.fft2(np.exp(1j * ph.astype(np.float64)))) ** 2
    np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-5 * float(want.max()))


@pytest.mark.gpu
def test_generic_incoming_amplitude_gs_and_gd(gpu, engine):
    """An incoming intensity (src/algorithms.py:14-19 / :65-70) on a shape with
    no radix plan: GS (uint8 target, warm start) and GD (float32 target, random
    guess scaled by a_in) against the faithful float64 oracle."""
    from spatial_light_modulator_module_amd import algorithms as alg

    shape = (90, 150)
    rng = np.random.default_rng(12)
    ain = np.sqrt(rng.uniform(0.25, 2.0, shape)).astype(np.float32)  # a_in; the oracle gets a_in^2 as the image
    inten = ain.astype(np.float64) ** 2
    t = _target(shape, True, seed=13)
    # SURVEY.md 8c warm-start protocol: the reference's phase after 30 cold iterations
    phi30, _, _ = orc.gerchberg_saxton_faithful(t, 30, incoming_intensity=inten)
    phi30 = phi30.astype(np.float32)
    ph, _, errs, _, _ = alg.run_gs(t[None], 30, ain=ain, initial_phase=phi30[None])
    ref, _, ref_err = orc.gerchberg_saxton_faithful(t, 30, incoming_intensity=inten, initial_phase=phi30)
    rms = orc.phase_rms(ph[0], ref)
    print(f"[parity] {engine} GS {shape} uint8 with a_in, warm 30+30: phase rms {rms:.3e}")
    assert rms < 1e-6
    np.testing.assert_allclose(errs[0], ref_err, rtol=1e-6)

    tf = _target(shape, False, seed=14)
    x0 = alg.make_initial_guess("random", inten ** 0.5, tf, 42)
    loops = 40
    ph, _, errs, _, _ = alg.run_gd(tf[None], loops, np.full(loops, 0.005), 1.0, ain=ain, initial_field=x0[None])
    ref, _, ref_err, _ = orc.gradient_descent_faithful(tf, loops, 0.005, 1.0, 0, incoming_intensity=inten,
                                                       initial_field=x0)
    rms = orc.phase_rms(ph[0], ref)
    print(f"[parity] {engine} GD {shape} with a_in, {loops} iterations: phase rms {rms:.3e}")
    assert rms < 1e-5  # the complex64 initial field crossing the C-ABI, as test_generic_gd_vs_oracle
    np.testing.assert_allclose(errs[0], ref_err, rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(1080, 1920), (1, 13), (26, 1), (77, 45), (1280, 1024), (8, 8192), (14, 35),
                                   (49, 20), (121, 169)])
def test_mixed_radix_fft2_c128_vs_numpy(gpu, shape):
    """slm_fft2_c128 (float64 in and out) on the mixed-radix kernels, every
    radix and the ragged / degenerate tiles, against numpy.fft at float64
    accuracy."""
    rng = np.random.default_rng(2)
    x = rng.standard_normal((2,) + shape) + 1j * rng.standard_normal((2,) + shape)
    for inverse in (False, True):
        got = gpu.fft2_c128(x, inverse=inverse)
        want = np.fft.ifft2(x) * (shape[0] * shape[1]) if inverse else np.fft.fft2(x)
        err = np.max(np.abs(got - want)) / np.max(np.abs(want))
        assert err < 1e-13, (shape, inverse, err)


@pytest.mark.gpu
def test_mixed_radix_gs_1080x1920_warm_start(gpu, monkeypatch):
    """A 1080 x 1920 SLM panel (1080 = 2^3 3^3 5, 1920 = 2^7 3 5) on the
    mixed-radix engine (float64; the default float32 run is
    test_gpu_radix_c64.py's), SURVEY.md 8c warm-start protocol (30 cold
    iterations of the faithful oracle, then 100 more) against the float64
    oracle."""
    import os

    import scipy.fft as sfft

    WORKERS = min(16, os.cpu_count() or 1)  # the GPU box gives a process a 16-CPU share

    monkeypatch.setenv("SLM_GENERIC_ENGINE", "mr")
    t = _target((1080, 1920), False, seed=21)
    with sfft.set_workers(WORKERS):
        phi30, _, _ = orc.gerchberg_saxton_faithful(t, 30)
        phi30 = phi30.astype(np.float32)
        ref, _, ref_err = orc.gerchberg_saxton_faithful(t, 100, initial_phase=phi30)
    with gpu.Plan(gpu.ALGO_GS, 1, 1080, 1920, gpu.TGT_F32, False, 100) as p:
        assert p.engine() == ("mixed-radix", "mixed-radix")
        p.set_target(t[None])
        p.set_phase(phi30[None])
        p.run(100)
        ph, _, stats, _ = p.read()
    rms = orc.phase_rms(ph[0], ref)
    print(f"[parity] mixed-radix GS 1080x1920 float32 target, warm 30+100: phase rms {rms:.3e}")
    assert rms < 1e-6
    np.testing.assert_allclose(stats[0, :100, 3], ref_err, rtol=1e-6)


@pytest.mark.gpu
def test_prime_side_runs_the_chirp_z_line_transforms(gpu, monkeypatch):
    """A side with a prime factor above 13 runs the line transforms (its own
    side by chirp-z, the other directly); 13-smooth shapes the mixed radix."""
    monkeypatch.delenv("SLM_GENERIC_ENGINE", raising=False)
    with gpu.Plan(gpu.ALGO_GS, 1, 97, 120, gpu.TGT_F32, False, 2) as p:
        assert p.engine() == ("bluestein", "bluestein")
    with gpu.Plan(gpu.ALGO_GS, 1, 99, 120, gpu.TGT_F32, False, 2) as p:
        assert p.engine() == ("mixed-radix", "mixed-radix")


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(97, 101), (1272, 96), (53, 1272)])
def test_prime_sides_gs_gd_vs_oracle(gpu, monkeypatch, shape):
    """Sides with a prime factor above 13 (97, 101; 1272 = 2^3 3 53) on the
    default engine: the chirp-z line transforms (Bluestein over a 5-smooth
    length >= 2n - 1, mr_line_kernel), O(N log N) like the reference's
    pocketfft (src/algorithms.py:27,31,34), against the faithful float64
    oracle -- GS by the SURVEY.md 8c warm start (30 + 30), GD from the random
    guess (30 iterations)."""
    from spatial_light_modulator_module_amd import algorithms as alg

    monkeypatch.delenv("SLM_GENERIC_ENGINE", raising=False)
    t = _target(shape, True, seed=31)
    phi30, _, _ = orc.gerchberg_saxton_faithful(t, 30)
    phi30 = phi30.astype(np.float32)
    ref, _, ref_err = orc.gerchberg_saxton_faithful(t, 30, initial_phase=phi30)
    ph, _, stats, _ = _gs(gpu, t[None], 30, phi30[None], engine="bluestein")
    rms = orc.phase_rms(ph[0], ref)
    tf = _target(shape, False, seed=32)
    x0 = alg.make_initial_guess("random", None, tf, 42)
    ref_gd, _, ref_gd_err, _ = orc.gradient_descent_faithful(tf, 30, 0.005, 1.0, 0, initial_field=x0)
    ph_gd, _, errs, _, _ = alg.run_gd(tf[None], 30, np.full(30, 0.005), 1.0, initial_field=x0[None])
    rms_gd = orc.phase_rms(ph_gd[0], ref_gd)
    print(f"[parity] bluestein {shape}: GS u8 warm 30+30 phase rms {rms:.3e}; GD 30 iterations {rms_gd:.3e}")
    assert rms < 1e-6
    np.testing.assert_allclose(stats[0, :30, 3], ref_err, rtol=1e-6)
    assert rms_gd < 1e-5  # the field crosses the C-ABI as complex64 (test_generic_gd_vs_oracle)
    np.testing.assert_allclose(errs[0], ref_gd_err, rtol=1e-5)
    alg.clear_plans()


@pytest.mark.gpu
def test_fft2_c128_integration_stub(gpu):
    """INTEGRATION.md's ctypes stub of slm_fft2_c128, as a maintainer would
    paste it, equals numpy.fft.ifft2 in float64 (src/move_traps.py:66)."""
    import ctypes

    _lib = ctypes.CDLL(gpu.LIB_PATH)
    _vp, _i = ctypes.c_void_p, ctypes.c_int
    _lib.slm_init.argtypes = [_i]
    _lib.slm_last_error.restype = ctypes.c_char_p
    _lib.slm_fft2_c128.argtypes = [_vp, _vp, _i, _i, _i, _i]

    def _p(a):
        return None if a is None else a.ctypes.data

    def ifft2_hip(x, device=0):
        if _lib.slm_init(device) != 0:
            raise RuntimeError(_lib.slm_last_error().decode())
        a = np.ascontiguousarray(x, np.complex128)
        out = np.empty_like(a)
        h, w = a.shape[-2:]
        if _lib.slm_fft2_c128(_p(a), _p(out), a.size // (h * w), h, w, 1) != 0:
            raise RuntimeError(_lib.slm_last_error().decode())
        return out / (h * w)

    img = np.zeros((768, 1024))
    img[5, 7] = 255.0
    img[300, 900] = 17.0
    np.testing.assert_allclose(ifft2_hip(img), np.fft.ifft2(img), rtol=0, atol=1e-15 * 255)
