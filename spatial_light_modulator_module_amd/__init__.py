"""MI355X-native drop-in for the GS / GD hologram loops of
pranislav/Spatial_Light_Modulator_Module (src/algorithms.py).

Compute runs only in libslm_hip.so (hand-written gfx950 HIP kernels, loaded
through ctypes by ``_lib.load()``). The library is loaded on first use by any
compute entry point and a missing build raises ImportError there: there is no
CPU fallback. The package imports no torch; pure host helpers (``parallel``)
can be imported without the library.
"""

__all__ = ["_lib", "algorithms", "parallel"]
