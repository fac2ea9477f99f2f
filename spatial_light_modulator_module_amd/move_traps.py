"""Trap holograms for the optical-tweezers loop, drop-in for the compute of
src/move_traps.py (the keyboard / Tk window plumbing around it is out of scope,
DESIGN.md section 7).

* ``update_hologram(black_image, coords, which)`` — src/move_traps.py:64-68:
  the phase of ``ifft2`` of a blank image with one 255-valued pixel, float64,
  computed on the GPU by slm_trap_frames (closed form of the single-pixel
  inverse DFT, exact integer phase index; no transform needed); an image that
  already holds traps takes the float64 device transform (slm_fft2_c128).
* ``hologram_frame(hologram, mask, mask_flag, ct2pi)`` — the quantisation of
  display_hologram, src/move_traps.py:135-139, as the uint8 frame handed to the
  SLM window.
* ``trap_frame(shape, coords, which, mask, mask_flag, ct2pi)`` — both fused in
  one launch: what a key press of the trap-moving loop costs.
"""
from __future__ import annotations

import numpy as np

from . import _lib


def _trap_index(black_image: np.ndarray, coords, which):
    h, w = black_image.shape
    y, x = int(coords[which][0]), int(coords[which][1])
    if not (-h <= y < h and -w <= x < w):  # numpy indexing rules of black_image[y][x]
        raise IndexError(f"index ({y}, {x}) is out of bounds for an image of shape {(h, w)}")
    return y % h, x % w


def update_hologram(black_image: np.ndarray, coords, which) -> np.ndarray:
    """src/move_traps.py:64-68: angle(ifft2(image with the trap pixel at 255)),
    float64; the pixel under the trap is left at 0 afterwards, as the reference
    leaves it. A blank image (the reference's loop, src/move_traps.py:16) takes
    the closed form (slm_trap_frames, exact phase index). Any other image runs
    the device's float64 inverse 2-D transform (slm_fft2_c128), as the
    reference's float64 ifft2 does (tests/test_frames.py)."""
    black_image = np.asarray(black_image)
    if black_image.ndim != 2:
        raise ValueError("black_image must be a 2-D image")
    y, x = _trap_index(black_image, coords, which)
    if not np.count_nonzero(black_image):
        phase, _ = _lib.trap_frames(black_image.shape, [y], [x], frame=False)
        black_image[y][x] = 0
        return phase[0]
    black_image[y][x] = 255
    # float64 on the device, as the reference's ifft2 of the float64 image (unscaled:
    # the 1/(h w) leaves angles alone)
    field = _lib.fft2_c128(black_image.astype(np.complex128), inverse=True)
    black_image[y][x] = 0
    return np.angle(field)


def hologram_frame(hologram: np.ndarray, mask, mask_flag: bool, ct2pi) -> np.ndarray:
    """uint8 SLM levels of display_hologram (src/move_traps.py:135-139):
    ((hologram [+ mask]) % 2pi * ct2pi / 2pi).astype(uint8)."""
    return _lib.quantize(np.asarray(hologram, dtype=np.float64), mask if mask_flag else None, ct2pi,
                         _lib.QUANT_ASTYPE)


def trap_frame(shape, coords, which, mask=None, mask_flag: bool = True, ct2pi=256):
    """update_hologram + display_hologram's quantisation in one launch; returns
    (hologram float64, frame uint8)."""
    y, x = _trap_index(np.empty(shape, np.uint8), coords, which)
    phase, frame = _lib.trap_frames(shape, [y], [x], mask if (mask_flag and mask is not None) else None, ct2pi,
                                    _lib.QUANT_ASTYPE)
    return phase[0], frame[0]
