"""Phase-mask correction of stored holograms, drop-in for
``mask_hologram(path, mask_arr, ct2pi)`` of src/display_holograms.py:253-266
(the display loop and its console commands are out of scope, DESIGN.md
section 7). The per-pixel arithmetic and the 8-bit conversion run on the GPU
(slm_quantize); the result is the same PIL 'L' image.
"""
from __future__ import annotations

import os

import numpy as np

from . import _lib


def mask_hologram(path, mask_arr, ct2pi):
    """.npy holograms: ((h + mask) % 2pi) / 2pi * ct2pi; images: (int16 image
    + mask / 2pi * ct2pi) % ct2pi; both through PIL's float -> 'L' conversion
    (clip to [0, 255], truncate)."""
    from PIL import Image

    if mask_arr is None:
        raise TypeError("mask_hologram needs a mask array (display_with_mask handles mask_arr=None)")
    mask = np.asarray(mask_arr, dtype=np.float64)
    base, ext = os.path.splitext(path)
    if ext == ".npy":
        hologram = np.load(path)
        out = _lib.quantize(np.asarray(hologram, dtype=np.float64), mask, ct2pi, _lib.QUANT_PIL)
    else:
        hologram = np.array(Image.open(path).convert("L")).astype(np.int16)
        out = _lib.quantize(hologram, mask, ct2pi)
    return Image.fromarray(out)  # uint8 -> mode 'L'
