#!/usr/bin/env python3
"""Relative l2 / max error of the GPU 2-D FFT and of scipy's complex64 FFT
against a float64 transform of the same (complex64) input."""
import os
import sys

import numpy as np
import scipy.fft as sfft

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatial_light_modulator_module_amd import _lib  # noqa: E402

_lib.init(0)
for n in (256, 1024, 4096):
    rng = np.random.default_rng(n)
    x = np.exp(1j * rng.uniform(-np.pi, np.pi, (n, n))).astype(np.complex64)
    ref = np.fft.fft2(x.astype(np.complex128))
    g = _lib.fft2(x).astype(np.complex128)
    c = sfft.fft2(x).astype(np.complex128)
    nr = np.linalg.norm(ref)
    print(f"n={n}: gpu rel_l2={np.linalg.norm(g-ref)/nr:.3e} max={np.abs(g-ref).max()/np.abs(ref).max():.3e} | "
          f"scipy c64 rel_l2={np.linalg.norm(c-ref)/nr:.3e} max={np.abs(c-ref).max()/np.abs(ref).max():.3e}")
    gi = _lib.fft2(x, inverse=True).astype(np.complex128)
    refi = np.fft.ifft2(x.astype(np.complex128)) * n * n
    print(f"       inverse gpu rel_l2={np.linalg.norm(gi-refi)/np.linalg.norm(refi):.3e}")
