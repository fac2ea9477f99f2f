"""GIF side paths and the float64-target rule of the drop-in.

* GD GIF frames (src/algorithms.py:94-101): chunked warm-started runs on the
  GPU vs the float64 oracle's field after the same iterations, frame by frame;
  the chunked run returns the same hologram as an unchunked one.
* GS GIF frames (src/algorithms.py:40-41, 52-57): frame names / count and the
  first frame vs the oracle (later cold-start frames are chaotic).
* float64 targets: max(T) and sum T^2 stay exact in float64
  (src/algorithms.py:21-23, :38, :161-162).
"""
import argparse
import os

import numpy as np
import pytest
from PIL import Image

from oracle import fast_f64
from oracle import gs_gd_oracle as orc


def _args(tmp_path, **kw):
    base = dict(incomming_intensity="uniform", tolerance=0.0, max_loops=7, gif=True, print_info=False,
                plot_error=False, learning_rate=0.005, white_attention=1.0, unsettle=0, initial_guess="random",
                random_seed=42, gif_type="h", gif_skip=2, gif_source_dir=str(tmp_path), correspond_to2pi=256)
    base.update(kw)
    return argparse.Namespace(**base)


def _frame(path):
    return np.array(Image.open(path), dtype=np.int16)


def _close_frames(got, want):
    """8-bit frames of phases that agree to ~1e-6 rad: equal but for a few
    pixels one level apart, or across the +-pi branch cut (0 <-> 255)."""
    d = np.abs(got - want)
    d = np.minimum(d, 256 - d)
    assert d.max() <= 1 and np.mean(d > 0) < 2e-3, (d.max(), np.mean(d > 0))


@pytest.mark.gpu
@pytest.mark.parametrize("gif_type,n", [("h", 64), ("i", 64), ("h", 1024)])
def test_gd_gif_frames_vs_oracle(gpu, tmp_path, gif_type, n):
    """n = 1024 runs the chunks on the configs[2] plan (narrow layout pair:
    the field read back and set again through that layout's relayouts)."""
    from spatial_light_modulator_module_amd.algorithms import gradient_descent

    rng = np.random.default_rng(4)
    t = rng.uniform(0, 255, (n, n)).astype(np.float32)
    a = _args(tmp_path, gif_type=gif_type, unsettle=1)
    holo, out, err = gradient_descent(t, a)
    assert len(err) == 7
    names = sorted(os.listdir(tmp_path))
    assert names == ["0.png", "1.png", "2.png", "3.png"]  # iterations 0, 2, 4, 6
    # oracle: the same schedule, field after iteration i
    rates, _ = orc.unsettle_schedule(0.005, 7, 1, 7)
    x = orc.make_initial_guess("random", np.ones(t.shape), t, 42)
    done = 0
    for k, i in enumerate((0, 2, 4, 6)):
        _, o_out, _, x = fast_f64.gradient_descent_f64(t, i + 1 - done, rates[done:i + 1], 1.0, initial_field=x)
        done = i + 1
        if gif_type == "h":
            img = Image.fromarray((np.angle(x / abs(x)) + np.pi) / (2 * np.pi) * 256)
        else:
            img = Image.fromarray(o_out)
        want = np.array(img.convert("L"), dtype=np.int16)
        _close_frames(_frame(tmp_path / f"{k}.png"), want)
    assert a.learning_rate == 0.005 * 2  # unsettle=1 doubles once by iteration 7 (round(7/2) = 4)
    # chunked == unchunked
    from spatial_light_modulator_module_amd.algorithms import gradient_descent as gd

    h2, o2, e2 = gd(t, _args(tmp_path, gif=False, unsettle=1))
    np.testing.assert_allclose(holo, h2, rtol=0, atol=1e-6)
    np.testing.assert_allclose(err, e2, rtol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("gif_type", ["h", "i"])
def test_gs_gif_frames(gpu, tmp_path, gif_type):
    """add_gif_image (src/algorithms.py:52-57): "h" frames are the phase of A,
    "i" frames the normalised expected_outcome |C|^2 norm / max (:36-37), both
    PIL 'L' images of the iteration's state."""
    from spatial_light_modulator_module_amd.algorithms import gerchberg_saxton

    rng = np.random.default_rng(8)
    t = rng.integers(0, 256, (128, 128)).astype(np.uint8)
    a = _args(tmp_path, gif_type=gif_type, max_loops=9, gif_skip=4)
    holo, exp, err = gerchberg_saxton(t, a)
    assert len(err) == 9
    assert sorted(os.listdir(tmp_path)) == ["0.png", "1.png", "2.png"]  # iterations 0, 4, 8
    ph1, exp1, err1 = orc.gerchberg_saxton_faithful(t, 1)
    if gif_type == "h":
        want = np.array(Image.fromarray((ph1 + np.pi) * 256 / (2 * np.pi)).convert("L"), dtype=np.int16)
        last = np.array(Image.fromarray((holo + np.pi) * 256 / (2 * np.pi)).convert("L"), dtype=np.int16)
    else:
        assert exp1.dtype == np.float64 and np.isclose(exp1.max(), t.max())
        want = np.array(Image.fromarray(exp1).convert("L"), dtype=np.int16)
        last = np.array(Image.fromarray(exp).convert("L"), dtype=np.int16)
    _close_frames(_frame(tmp_path / "0.png"), want)
    np.testing.assert_allclose(err[0], err1[0], rtol=1e-5)
    # the last frame is the image of the returned hologram / expected outcome
    np.testing.assert_array_equal(_frame(tmp_path / "2.png"), last)


@pytest.mark.gpu
def test_float64_target_keeps_exact_stats(gpu):
    from spatial_light_modulator_module_amd import algorithms as alg

    rng = np.random.default_rng(64)
    t = rng.uniform(0, 255, (128, 128))  # float64, not representable in float32
    phi0 = rng.uniform(-np.pi, np.pi, t.shape).astype(np.float32)
    phase, e, errs, norm, emax = alg.run_gs(t[None], 8, initial_phase=phi0[None])
    assert norm[0] == np.amax(t)
    plan = alg.get_plan(alg.ALGO_GS, 1, 128, 128, alg.TGT_F32, False, 8)
    n2, s2 = plan.target_stats()
    assert n2[0] == np.amax(t) and s2[0] == np.einsum("ij,ij->", t, t)
    ph_o, exp_o, err_o = orc.gerchberg_saxton_faithful(t, 8, initial_phase=phi0)
    np.testing.assert_allclose(errs[0], err_o, rtol=2e-6)
    assert orc.phase_rms(phase[0], ph_o) < 1e-5
    np.testing.assert_allclose(alg.expected_from(e[0], norm[0], emax[0]), exp_o, rtol=1e-3, atol=1e-3 * norm[0])
