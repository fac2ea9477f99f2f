"""Pin the CPU oracle to the reference's own outputs (tests/golden/*.npz).

The goldens were produced by tests/golden/make_goldens.py, which imports the
reference's src/algorithms.py. The faithful oracle must reproduce them to
rounding level; the complex64 model (the GPU's arithmetic) must stay inside the
float32 band measured in SURVEY.md section 8c.
"""
import os

import numpy as np
import pytest

from oracle import gs_gd_oracle as orc


def load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


@pytest.mark.parametrize("name", ["g1_gs_u8_256.npz", "g2_gs_f32_256.npz"])
def test_gs_faithful_cold_and_warm(golden_dir, name):
    g = load(golden_dir, name)
    t = g["target"]
    phi30, _, err30 = orc.gerchberg_saxton_faithful(t, 30)
    np.testing.assert_allclose(phi30, g["phi30"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(err30, g["err30"], rtol=1e-12)
    # warm start: the loop state is angle(A) only (checkpoint/resume)
    phi, exp, err = orc.gerchberg_saxton_faithful(t, 200, initial_phase=g["phi30"])
    np.testing.assert_allclose(phi, g["phi230"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(err, g["err230"][30:], rtol=1e-12)
    np.testing.assert_allclose(exp.astype(np.float32), g["expected230"], rtol=1e-6)


def test_gs_faithful_traps(golden_dir):
    g = load(golden_dir, "g3_gs_traps_128.npz")
    phi, exp, err = orc.gerchberg_saxton_faithful(g["target"], 20)
    np.testing.assert_allclose(phi, g["phi"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(exp, g["expected"], rtol=1e-12, atol=1e-9)
    np.testing.assert_allclose(err, g["err"], rtol=1e-12)


def test_gs_faithful_incoming_intensity(golden_dir):
    from PIL import Image

    g = load(golden_dir, "g8_gs_ain_128.npz")
    img = np.array(Image.open(os.path.join(golden_dir, "g8_incoming_128.png")))
    phi, exp, err = orc.gerchberg_saxton_faithful(g["target"], 40, incoming_intensity=img)
    np.testing.assert_allclose(phi, g["phi40"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(err, g["err40"], rtol=1e-12)
    phi_w, _, err_w = orc.gerchberg_saxton_faithful(g["target"], 30, incoming_intensity=img,
                                                    initial_phase=g["phi10"])
    np.testing.assert_allclose(phi_w, g["phi40"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(err_w, g["err40"][10:], rtol=1e-12)


def test_gd_faithful(golden_dir):
    g = load(golden_dir, "g4_gd_f32_256.npz")
    phi, out, err, lr = orc.gradient_descent_faithful(g["target"], 100, 0.005, 1.0, 0, random_seed=42)
    np.testing.assert_allclose(phi, g["phi100"], rtol=0, atol=1e-10)
    np.testing.assert_allclose(err, g["err100"], rtol=1e-12)
    np.testing.assert_allclose(out.astype(np.float32), g["output100"], rtol=1e-6, atol=1e-3)
    assert lr == 0.005


def test_gd_faithful_fourier_unsettle(golden_dir):
    g = load(golden_dir, "g9_gd_fourier_u8_128.npz")
    phi, out, err, lr = orc.gradient_descent_faithful(g["target"], 60, 0.002, 2.0, 1, initial_guess="fourier")
    np.testing.assert_allclose(phi, g["phi"], rtol=0, atol=1e-10)
    np.testing.assert_allclose(err, g["err"], rtol=1e-12)
    assert lr == float(g["lr_after"])


def test_probes(golden_dir):
    g = load(golden_dir, "g6_probes.npz")
    # np.sqrt(uint8) is float16 = float16(sqrtf(x))
    assert str(g["sqrt_u8_dtype"]) == "float16"
    x = np.arange(256, dtype=np.float32)
    np.testing.assert_array_equal(np.sqrt(x).astype(np.float16), g["sqrt_u8"])
    # Python's random stream == RandomState([seed]).random_sample
    np.testing.assert_array_equal(orc.random_unit_draws(42, 4096), g["py_random_42"])
    z = np.zeros((16, 16))
    np.testing.assert_array_equal(orc.make_initial_guess("random", np.ones((16, 16)), z, 42), g["guess_random_16"])
    z8 = np.zeros((8, 8))
    for k in ("old", "unnormed", "zeros", "ones"):
        np.testing.assert_array_equal(orc.make_initial_guess(k, np.ones((8, 8)), z8, 7), g[f"guess_{k}_8"])


def test_edges(golden_dir):
    g = load(golden_dir, "g7_edges.npz")
    assert str(g["gs_zero_loops"]) == "UnboundLocalError"
    assert str(g["gd_bad_guess"]) == "ValueError"
    with pytest.raises(UnboundLocalError):
        orc.gerchberg_saxton_faithful(np.ones((8, 8), np.uint8), 0)
    with pytest.raises(ValueError):
        orc.make_initial_guess("bogus", np.ones((4, 4)), np.zeros((4, 4)), 1)
    # all-zero target: error 0 after the first loop ends the run (while error > 0)
    _, _, errz = orc.gerchberg_saxton_faithful(np.zeros((64, 64), np.uint8), 5)
    np.testing.assert_array_equal(errz, g["zeros_target_err"])
    assert len(errz) == 1
    _, lr = orc.unsettle_schedule(0.005, 4, 1, 4)
    assert lr == float(g["unsettle_lr_after"])
    t3 = load(golden_dir, "g3_gs_traps_128.npz")["target"]
    _, _, err_tol = orc.gerchberg_saxton_faithful(t3, 60, tolerance=1e9)
    np.testing.assert_allclose(err_tol, g["tol_hit_err"], rtol=1e-12)


def test_c64_model_within_float32_band(golden_dir):
    """The GPU's arithmetic model stays inside the float32 band of SURVEY 8c
    (warm start phi30 -> +200 iterations: measured 3.8e-6 / 6.5e-6 rms)."""
    for name in ("g1_gs_u8_256.npz", "g2_gs_f32_256.npz"):
        g = load(golden_dir, name)
        phi, _, stats = orc.gerchberg_saxton_c64(g["target"], 200, initial_phase=g["phi30"])
        assert orc.phase_rms(phi, g["phi230"]) < 1e-5
        t = g["target"].astype(np.float64)
        err = orc.error_from_stats(stats, t.max(), np.sum(t * t), t.size)
        np.testing.assert_allclose(err, g["err230"][30:], rtol=1e-4)


def test_error_expansion_matches_direct():
    rng = np.random.default_rng(0)
    t = rng.uniform(0, 255, (64, 64))
    e = rng.uniform(0, 1e9, (64, 64))
    direct = orc.error_f(e * (t.max() / e.max()), t, t.size)
    stats = np.array([e.max(), np.sum(e * e), np.sum(e * t)])
    np.testing.assert_allclose(orc.error_from_stats(stats, t.max(), np.sum(t * t), t.size), direct, rtol=1e-9)


# ---------------------------------------------------------------------------
# the multi-threaded float64 restatements (oracle/fast_f64.py) used by the
# large-size GPU gates: pinned to the reference goldens and the faithful path
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["g1_gs_u8_256.npz", "g2_gs_f32_256.npz"])
def test_fast_gs_warm_start_matches_reference(golden_dir, name):
    from oracle import fast_f64

    g = load(golden_dir, name)
    phi, exp, err = fast_f64.gerchberg_saxton_f64(g["target"], 200, initial_phase=g["phi30"], workers=4)
    # z/|z| in place of exp(1j angle z): rounding-level differences only
    assert orc.phase_rms(phi, g["phi230"]) < 1e-12
    np.testing.assert_allclose(err, g["err230"][30:], rtol=1e-11)
    np.testing.assert_allclose(exp.astype(np.float32), g["expected230"], rtol=1e-5)


def test_fast_gs_incoming_intensity_and_tolerance(golden_dir):
    from PIL import Image

    from oracle import fast_f64

    g = load(golden_dir, "g8_gs_ain_128.npz")
    # float64 intensity: with the uint8 PNG itself np.sqrt gives float16 and the
    # reference's whole loop runs in complex64 (the faithful restatement and the
    # g8 golden cover that dtype flow); the fast oracle is the float64 model
    img = np.array(Image.open(os.path.join(golden_dir, "g8_incoming_128.png"))).astype(np.float64)
    phi, _, err = fast_f64.gerchberg_saxton_f64(g["target"], 30, initial_phase=g["phi10"], incoming_intensity=img,
                                                workers=2)
    ref_phi, _, ref_err = orc.gerchberg_saxton_faithful(g["target"], 30, incoming_intensity=img,
                                                        initial_phase=g["phi10"])
    assert orc.phase_rms(phi, ref_phi) < 1e-12
    np.testing.assert_allclose(err, ref_err, rtol=1e-11)
    t3 = load(golden_dir, "g3_gs_traps_128.npz")["target"]
    _, _, err_tol = fast_f64.gerchberg_saxton_f64(t3, 60, tolerance=1e9, workers=2)
    assert len(err_tol) == len(load(golden_dir, "g7_edges.npz")["tol_hit_err"])


def test_fast_gd_matches_reference(golden_dir):
    from oracle import fast_f64

    g = load(golden_dir, "g4_gd_f32_256.npz")
    t = g["target"]
    x0 = orc.make_initial_guess("random", np.ones(t.shape), t, 42)
    phi, out, err, x = fast_f64.gradient_descent_f64(t, 100, 0.005, 1.0, initial_field=x0, workers=4)
    assert orc.phase_rms(phi, g["phi100"]) < 1e-11
    np.testing.assert_allclose(err, g["err100"], rtol=1e-11)
    np.testing.assert_allclose(out.astype(np.float32), g["output100"], rtol=1e-5, atol=1e-3)
    # continuing from the returned field reproduces one long run
    phi5, _, err5, _ = fast_f64.gradient_descent_f64(t, 400, 0.005, 1.0, initial_field=x, workers=4)
    np.testing.assert_allclose(np.concatenate([err, err5]), g["err500"], rtol=1e-9)
    assert orc.phase_rms(phi5, g["phi500"]) < 1e-6  # the golden phi500 is stored as float32


def test_fast_gd_unsettle_schedule_matches_faithful():
    from oracle import fast_f64

    rng = np.random.default_rng(5)
    t = rng.integers(0, 256, (64, 64)).astype(np.uint8)
    rates, lr_after = orc.unsettle_schedule(0.003, 30, 2, 30)
    x0 = orc.make_initial_guess("random", np.ones(t.shape), t, 9)
    phi, _, err, _ = fast_f64.gradient_descent_f64(t, 30, rates, 1.5, initial_field=x0, workers=1)
    ref_phi, _, ref_err, ref_lr = orc.gradient_descent_faithful(t, 30, 0.003, 1.5, 2, random_seed=9)
    assert lr_after == ref_lr
    assert orc.phase_rms(phi, ref_phi) < 1e-11
    np.testing.assert_allclose(err, ref_err, rtol=1e-11)
