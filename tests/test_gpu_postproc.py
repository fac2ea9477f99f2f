"""GPU post-processing of the hologram CLI against the
reference's per-pixel loops, restated here verbatim in Python:

* deflect_2pi  src/wavefront_correction.py:440-449
* lens         src/generate_hologram.py:189-203 (uint8 storage)
* deflect_hologram / add_lens / transform_hologram  src/generate_hologram.py:82-87,178-186
* show_expected_outcome's |fft2(exp(1j h))|^2      src/generate_hologram.py:24-34

The kernel (slm_transform_hologram) keeps the reference's float64 operation
order with no contraction, so holograms and lens levels match bit for bit.
"""
import os

import numpy as np
import pytest

from spatial_light_modulator_module_amd import constants as c


def ref_deflect_2pi(angle):
    x_angle, y_angle = angle
    hologram = np.zeros((c.slm_height, c.slm_width))
    const = 2 * np.pi * c.px_distance / c.wavelength
    for i in range(c.slm_height):
        for j in range(c.slm_width):
            new_phase = const * (np.sin(y_angle * c.u) * i + np.sin(x_angle * c.u) * j)
            hologram[i, j] = new_phase % (2 * np.pi)
    return hologram


def ref_lens(focal_length, shape):
    h, w = shape
    hologram = np.zeros((h, w), dtype=np.uint8)
    for i in range(h):
        for j in range(w):
            r = c.px_distance * np.sqrt((i - h / 2) ** 2 + (j - w / 2) ** 2)
            phase_shift = 2 * np.pi * focal_length / c.wavelength * (1 - np.sqrt(1 + r**2 / focal_length**2))
            hologram[i, j] = phase_shift % (2 * np.pi)
    return hologram


@pytest.mark.gpu
@pytest.mark.timeout(300)
@pytest.mark.parametrize("angle,focal", [((1.0, 0.5), 2.0), ((-2.0, 3.0), -0.7)])
def test_transform_bitwise_vs_reference_loops(gpu, angle, focal):
    from spatial_light_modulator_module_amd import generate_hologram as gh

    rng = np.random.default_rng(7)
    holo = rng.uniform(-np.pi, np.pi, (c.slm_height, c.slm_width))
    shape = holo.shape
    ramp = ref_deflect_2pi(angle)
    levels = ref_lens(focal, shape)
    # deflect alone on the analytical (zero) hologram: the ramp itself
    np.testing.assert_array_equal(gpu.transform_hologram(None, *shape, gh.deflect_params(angle)), ramp % (2 * np.pi))
    # lens alone: the uint8 levels, as (0 + level) % 2pi
    got = gpu.transform_hologram(None, *shape, None, gh.lens_params(focal))
    np.testing.assert_array_equal(got, levels.astype(np.float64) % (2 * np.pi))
    # transform_hologram(h, deflect + lens) of the reference
    want = ((holo + ramp) % (2 * np.pi) + levels) % (2 * np.pi)
    got = gpu.transform_hologram(holo, *shape, gh.deflect_params(angle), gh.lens_params(focal))
    np.testing.assert_array_equal(got, want)
    assert np.abs(got - want).max() <= 1e-12


@pytest.mark.gpu
def test_analytical_hologram_cli(gpu, tmp_path, monkeypatch):
    from spatial_light_modulator_module_amd import generate_hologram as gh

    monkeypatch.chdir(tmp_path)
    path = gh.cli(["-deflect", "1", "0.5", "-lens", "2.0", "-dest_dir", "out"])
    assert os.path.basename(path) == "analytical_deflect_x1.0_y0.5_lens2.0.npy"
    h = np.load(path)
    want = (ref_deflect_2pi((1.0, 0.5)) % (2 * np.pi) + ref_lens(2.0, h.shape)) % (2 * np.pi)
    np.testing.assert_array_equal(h, want)
    # the vectorised host twins agree too
    np.testing.assert_array_equal(h, gh.add_lens(gh.deflect_hologram(np.zeros(h.shape), (1.0, 0.5)), 2.0))
    path2 = gh.cli(["-deflect", "1", "0.5", "-lens", "2.0", "-dest_dir", "out"])
    assert path2.endswith("analytical_deflect_x1.0_y0.5_lens2.0_1.npy")


@pytest.mark.gpu
@pytest.mark.parametrize("shape", [(768, 1024), (256, 256)])
def test_preview_intensity_vs_numpy(gpu, shape):
    from spatial_light_modulator_module_amd import generate_hologram as gh

    rng = np.random.default_rng(11)
    holo = rng.uniform(0, 2 * np.pi, shape)
    want = np.abs(np.fft.fft2(np.exp(1j * holo))) ** 2
    want = want / np.amax(want) * 200
    got = gh.expected_outcome_image(holo, 200)
    assert got.dtype == np.float64 and got.shape == shape
    # complex64 transform of a float32 phase: relative to the peak
    np.testing.assert_allclose(got, want, rtol=0, atol=2e-4 * 200)
