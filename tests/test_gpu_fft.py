"""2-D transform kernels (row + column passes) against numpy's FFT.

The reference's transforms are scipy.fft.fft2 / ifft2 (src/algorithms.py:27,31,
34,84,88); the library's are unscaled in both directions.
"""
import numpy as np
import pytest

SHAPES = [(64, 64), (128, 256), (256, 256), (512, 128), (768, 1024), (1024, 1024), (2048, 256), (256, 2048),
          (4096, 64), (64, 4096), (1024, 768)]


@pytest.mark.gpu
@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("inverse", [False, True])
def test_fft2_matches_numpy(gpu, shape, inverse):
    rng = np.random.default_rng(hash(shape) % 2**32)
    x = (rng.standard_normal((2,) + shape) + 1j * rng.standard_normal((2,) + shape)).astype(np.complex64)
    got = gpu.fft2(x, inverse=inverse).astype(np.complex128)
    ref = np.fft.ifft2(x.astype(np.complex128)) * (shape[0] * shape[1]) if inverse else np.fft.fft2(
        x.astype(np.complex128))
    err = np.linalg.norm(got - ref) / np.linalg.norm(ref)
    # float32 FFT: relative l2 error ~ eps * sqrt(log2 N)
    assert err < 2e-6, f"relative error {err:.3e}"


@pytest.mark.gpu
def test_fft2_roundtrip_large(gpu):
    rng = np.random.default_rng(7)
    x = (rng.standard_normal((4096, 4096)) + 1j * rng.standard_normal((4096, 4096))).astype(np.complex64)
    y = gpu.fft2(gpu.fft2(x), inverse=True) / (4096 * 4096)
    err = np.linalg.norm(y - x) / np.linalg.norm(x)
    assert err < 2e-6, f"round trip error {err:.3e}"


@pytest.mark.gpu
@pytest.mark.parametrize("variant", ["wide", "narrow"])
@pytest.mark.parametrize("shape", [(256, 512), (768, 1024), (1024, 2048)])
def test_fft2_plan_variants(gpu, monkeypatch, variant, shape):
    """Both radix-plan variants (wide: 16-24 elements per thread; narrow: half)
    compute the same transform."""
    monkeypatch.setenv("SLM_PLAN", variant)
    rng = np.random.default_rng(3)
    x = (rng.standard_normal(shape) + 1j * rng.standard_normal(shape)).astype(np.complex64)
    got = gpu.fft2(x).astype(np.complex128)
    ref = np.fft.fft2(x.astype(np.complex128))
    assert np.linalg.norm(got - ref) / np.linalg.norm(ref) < 2e-6
