"""SLM frame path: single-trap holograms
(src/move_traps.py:64-68), display quantisation (src/move_traps.py:135-139) and
mask correction of stored holograms (src/display_holograms.py:253-266).

CPU tests pin the oracle restatement (oracle/frames_oracle.py) to independent
facts (the plane-wave form of a single-pixel inverse DFT, the installed PIL's
float -> 'L' rule) and the host-side argument handling; GPU tests compare the
HIP kernels with the oracle. Phases are floating point: wrapped difference
<= 1e-12 rad. Levels are integers: identical, except pixels whose value
before truncation lies within 1e-9 of an integer level (a 1-ulp difference in
the phase can legitimately move those across the boundary); those are counted
and must be rare when a random mask is added (bare trap phases are exact
multiples of 2 pi / S, so many of their levels sit on a boundary: there the
level follows the last ulp of pocketfft's phase and cannot be pinned).
"""
import os

import numpy as np
import pytest

from oracle import frames_oracle as fo

SHAPES = [(768, 1024), (64, 128), (256, 256)]
TRAPS = [(0, 0), (1, 0), (0, 1), (383, 511), (767, 1023), (200, 700), (-1, -5)]


def wrapped(a, b):
    return np.abs(np.angle(np.exp(1j * (np.asarray(a) - np.asarray(b)))))


def near_level(v, tol=1e-9):
    v = np.asarray(v, np.float64)
    return np.abs(v - np.round(v)) < tol


# ---------------------------------------------------------------- CPU -----
@pytest.mark.parametrize("shape", SHAPES)
def test_oracle_update_hologram_is_a_plane_wave(shape):
    """angle(ifft2(delta)) = 2 pi (k y / H + l x / W) wrapped: the closed form
    the HIP kernel evaluates (frames.hip)."""
    h, w = shape
    for y, x in [(0, 0), (3, 5), (h - 1, w - 1)]:
        img = np.zeros(shape, np.uint8)
        ph = fo.update_hologram(img, [[y, x]], 0)
        k = np.arange(h)[:, None]
        l = np.arange(w)[None, :]
        want = 2 * np.pi * (((k * y) % h) / h + ((l * x) % w) / w)
        assert wrapped(ph, want).max() < 1e-12
        assert not img.any()  # the reference resets the pixel


def test_pil_float_to_l_rule_is_clip_and_truncate():
    """The rule slm_quantize implements for PIL (frames.hip pil_f_to_l)."""
    from PIL import Image

    v = np.array([[0.2, 0.7, 1.5, 2.999, 254.6, 255.4, 300.0, -1.0, -0.4, 127.5]])
    got = np.array(Image.fromarray(v).convert("L"))
    want = np.clip(np.trunc(v.astype(np.float32)), 0, 255).astype(np.uint8)
    np.testing.assert_array_equal(got, want)


def test_update_hologram_argument_checks():
    from spatial_light_modulator_module_amd import move_traps as mt

    with pytest.raises(IndexError):
        mt._trap_index(np.zeros((4, 4)), [[4, 0]], 0)
    assert mt._trap_index(np.zeros((4, 6)), [[-1, -2]], 0) == (3, 4)


# ---------------------------------------------------------------- GPU -----
@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES)
def test_trap_phase_matches_reference(gpu, shape):
    from spatial_light_modulator_module_amd import move_traps as mt

    h, w = shape
    for y, x in TRAPS:
        if not (-h <= y < h and -w <= x < w):
            continue
        ref = fo.update_hologram(np.zeros(shape, np.uint8), [[y, x]], 0)
        img = np.zeros(shape, np.uint8)
        got = mt.update_hologram(img, [[0, 0], [y, x]], 1)
        assert got.dtype == np.float64 and got.shape == shape
        assert wrapped(got, ref).max() < 1e-12, (y, x)
        assert not img.any()


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(256, 256), (768, 1024), (90, 150)])
def test_update_hologram_non_blank(gpu, shape):
    """An image already holding traps (src/move_traps.py:64-68 with a non-blank
    black_image): angle(ifft2) through the device's float64 transform
    (slm_fft2_c128) vs the float64 reference restatement at EVERY pixel --
    the SLM shows the phase wherever the field is dim too."""
    from spatial_light_modulator_module_amd import move_traps as mt

    rng = np.random.default_rng(11)
    img = np.zeros(shape, np.uint8)
    img[rng.integers(0, shape[0], 5), rng.integers(0, shape[1], 5)] = rng.integers(1, 256, 5)
    y, x = 7, shape[1] - 3
    want_img = img.copy()
    ref = fo.update_hologram(want_img, [[y, x]], 0)
    lit = img.astype(np.float64)
    lit[y, x] = 255
    field = np.fft.ifft2(lit)
    # a float64 transform's angle error is ~1e-16 max|field| / |field|: every pixel
    # whose field is not itself at rounding level (none of these images has one)
    keep = np.abs(field) > 1e-9 * np.abs(field).max()
    got = mt.update_hologram(img, [[y, x]], 0)
    assert got.dtype == np.float64 and got.shape == shape
    err = wrapped(got, ref)[keep].max()
    print(f"[parity] non-blank update_hologram {shape}: max wrapped phase error {err:.2e} on {keep.mean():.6f} "
          f"of pixels (smallest |field| / max {np.abs(field).min() / np.abs(field).max():.2e})")
    assert keep.mean() > 0.999 and err < 1e-6
    np.testing.assert_array_equal(img, want_img)  # the trap pixel is back at 0, the rest untouched


@pytest.mark.gpu
def test_trap_phase_4096(gpu):
    from spatial_light_modulator_module_amd import _lib

    ys, xs = [4095, 1234], [17, 4000]
    ph, _ = _lib.trap_frames((4096, 4096), ys, xs, frame=False)
    for b, (y, x) in enumerate(zip(ys, xs)):
        ref = fo.update_hologram(np.zeros((4096, 4096), np.uint8), [[y, x]], 0)
        assert wrapped(ph[b], ref).max() < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("mask_flag", [False, True])
@pytest.mark.parametrize("ct2pi", [256, 200, 177.5])
def test_display_levels_match_reference(gpu, mask_flag, ct2pi):
    from spatial_light_modulator_module_amd import move_traps as mt

    rng = np.random.default_rng(7)
    shape = (768, 1024)
    mask = rng.uniform(-7, 7, shape)
    for y, x in [(0, 0), (100, 300), (767, 1)]:
        ref_h = fo.update_hologram(np.zeros(shape, np.uint8), [[y, x]], 0)
        ref = fo.display_levels(ref_h, mask, mask_flag, ct2pi)
        pre = fo.display_prequant(ref_h, mask, mask_flag, ct2pi)
        # quantisation of a given hologram: bit-exact
        got = mt.hologram_frame(ref_h, mask, mask_flag, ct2pi)
        np.testing.assert_array_equal(got, ref)
        # fused trap + quantisation: identical away from level boundaries
        ph, fr = mt.trap_frame(shape, [[y, x]], 0, mask, mask_flag, ct2pi)
        assert wrapped(ph, ref_h).max() < 1e-12
        diff = fr != ref
        edge = near_level(pre) | (np.abs(pre - ct2pi) < 1e-9)  # a level boundary or the 2 pi wrap
        assert not np.any(diff & ~edge), "level mismatch away from a boundary"
        if mask_flag:  # random masks put few values on a boundary; bare traps put many (exact multiples of 2 pi / S)
            assert diff.sum() <= 16


@pytest.mark.gpu
@pytest.mark.parametrize("ct2pi", [256, 220])
def test_mask_hologram_npy_and_image(gpu, tmp_path, ct2pi):
    from PIL import Image

    from spatial_light_modulator_module_amd import display_holograms as dh

    rng = np.random.default_rng(11)
    shape = (768, 1024)
    mask = rng.uniform(0, 2 * np.pi, shape)
    npy = os.path.join(tmp_path, "holo.npy")
    np.save(npy, rng.uniform(-np.pi, np.pi, shape))
    png = os.path.join(tmp_path, "holo.png")
    Image.fromarray(rng.integers(0, 256, shape).astype(np.uint8)).save(png)
    for path in (npy, png):
        got = dh.mask_hologram(path, mask, ct2pi)
        ref = fo.mask_hologram(path, mask, ct2pi)
        assert got.mode == "L" and got.size == ref.size
        np.testing.assert_array_equal(np.array(got), np.array(ref))
