#!/usr/bin/env python3
"""Forward/inverse 2-D FFT of the library (slm_fft2) against numpy for column
tile widths and sizes: python tools/diag_fft.py 1024x4:4,8,16 4096x1:0"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spatial_light_modulator_module_amd import _lib  # noqa: E402


def main():
    _lib.init(0)
    for spec in sys.argv[1:]:
        shape, cws = spec.split(":")
        n, b = (int(v) for v in shape.split("x"))
        rng = np.random.default_rng(n)
        x = (rng.standard_normal((b, n, n)) + 1j * rng.standard_normal((b, n, n))).astype(np.complex64)
        ref = np.fft.fft2(x.astype(np.complex128))
        refi = np.fft.ifft2(x.astype(np.complex128)) * (n * n)
        for cw in cws.split(","):
            if cw != "0":
                os.environ["SLM_COL_CW"] = cw
            else:
                os.environ.pop("SLM_COL_CW", None)
            y = _lib.fft2(x)
            yi = _lib.fft2(x, inverse=True)
            e = np.abs(y - ref).max() / np.abs(ref).max()
            ei = np.abs(yi - refi).max() / np.abs(refi).max()
            print(f"{shape} cw={cw}: fwd max rel {e:.2e} inv {ei:.2e}", flush=True)


if __name__ == "__main__":
    main()
