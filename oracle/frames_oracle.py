"""CPU oracle for the SLM frame path — TEST INFRASTRUCTURE ONLY.

Only tests/ may import this module, as the checker. Restatements of
pranislav/Spatial_Light_Modulator_Module (snapshot 2024-10-08), with the same
NumPy / SciPy / PIL operations in the same order as the reference:

* update_hologram   src/move_traps.py:64-68
* display_hologram  src/move_traps.py:135-139 (its quantisation; the Tk display is UI)
* mask_hologram     src/display_holograms.py:253-266

src/move_traps.py imports ``keyboard`` (not installed here), so the functions
are restated rather than imported; the PIL float -> 'L' rule is the installed
Pillow's own (Pillow 12.2 here; the reference pins 10.3): parity is pinned
against this Pillow, not the pinned one.
"""
from __future__ import annotations

import os

import numpy as np
from scipy.fft import ifft2


def update_hologram(black_image, coords, which):
    """src/move_traps.py:64-68."""
    black_image[coords[which][0]][coords[which][1]] = 255
    hologram = np.angle(ifft2(black_image))
    black_image[coords[which][0]][coords[which][1]] = 0
    return hologram


def display_levels(hologram, mask, mask_flag, ct2pi):
    """The uint8 image display_hologram hands to the window, src/move_traps.py:135-139."""
    if mask_flag:
        hologram = hologram + mask
    return (hologram % (2 * np.pi) * ct2pi / (2 * np.pi)).astype(np.uint8)


def display_prequant(hologram, mask, mask_flag, ct2pi):
    """The float64 value display_levels truncates (for boundary accounting)."""
    if mask_flag:
        hologram = hologram + mask
    return hologram % (2 * np.pi) * ct2pi / (2 * np.pi)


def mask_hologram(path, mask_arr, ct2pi):
    """src/display_holograms.py:253-266 (returns the PIL image)."""
    import PIL.Image as im

    base, ext = os.path.splitext(path)
    if ext == ".npy":
        hologram_arr_2pi = np.load(path)
        corrected_hologram_arr_2pi = (hologram_arr_2pi + mask_arr) % (2 * np.pi)
        corrected_hologram_arr = corrected_hologram_arr_2pi / (2 * np.pi) * ct2pi
    else:
        hologram_im = im.open(path).convert("L")
        hologram_arr = np.array(hologram_im).astype(np.int16)
        corrected_hologram_arr = (hologram_arr + (mask_arr / (2 * np.pi) * ct2pi)) % ct2pi
    corrected_hologram_im = im.fromarray(corrected_hologram_arr).convert("L")
    return corrected_hologram_im


def mask_prequant(path, mask_arr, ct2pi):
    """The float value mask_hologram hands to PIL (for boundary accounting)."""
    import PIL.Image as im

    base, ext = os.path.splitext(path)
    if ext == ".npy":
        return ((np.load(path) + mask_arr) % (2 * np.pi)) / (2 * np.pi) * ct2pi
    arr = np.array(im.open(path).convert("L")).astype(np.int16)
    return (arr + (mask_arr / (2 * np.pi) * ct2pi)) % ct2pi
