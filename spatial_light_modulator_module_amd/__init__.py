"""MI355X-native drop-in for the GS / GD hologram loops of
pranislav/Spatial_Light_Modulator_Module (src/algorithms.py).

Compute runs only in libslm_hip.so (hand-written gfx950 HIP kernels, loaded
through ctypes); importing this package loads that library eagerly so that a
missing build fails at import time rather than silently later.
"""
from . import _lib

_lib.load()

__all__ = ["_lib"]
