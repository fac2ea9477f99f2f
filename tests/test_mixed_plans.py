"""CPU check of the mixed-E Stockham pass arithmetic (csrc/radix_c128.hpp
mx_from, csrc/plans.hpp ep[]) through its NumPy model against numpy.fft."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))

import numpy as np  # noqa: E402

import mixed_plan_model as mpm  # noqa: E402


def test_every_mixed_plan_matches_numpy():
    plans = list(mpm.mixed_plans())
    assert {n for n, _, _ in plans} >= {600, 800, 1080, 1152, 1200, 1280, 1536, 1920}
    rng = np.random.default_rng(5)
    for n, r, ep in plans:
        assert int(np.prod(r)) == n
        x = rng.standard_normal(n) + 1j * rng.standard_normal(n)
        np.testing.assert_allclose(mpm.stockham(x, r, ep, False), np.fft.fft(x), atol=1e-9)
        np.testing.assert_allclose(mpm.stockham(x, r, ep, True), np.fft.ifft(x) * n, atol=1e-9)
        # the pass with the fewest elements sets the line's thread count (plans.hpp e)
        assert all(n % e == 0 and e % rr == 0 for rr, e in zip(r, ep))
