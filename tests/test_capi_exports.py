"""The C-ABI library loads on a GPU-less host and exports every entry point
include/slm_hip.h declares (no compute calls: there is no device here)."""
import ctypes
import os
import re
import subprocess

from spatial_light_modulator_module_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "slm_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(slm_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("slm_plan_create", "slm_plan_run", "slm_plan_read", "slm_gs", "slm_gd", "slm_fft2",
              "slm_plan_gather_phase"):
        assert s in syms
    assert len(syms) >= 25


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, f"declared in slm_hip.h but not exported: {missing}"


def test_exports_are_c_linkage():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert set(declared_symbols()) <= exported


def test_python_binding_covers_the_header():
    # every header function has a ctypes prototype in _lib (argtypes set)
    lib = _lib.load()
    for s in declared_symbols():
        assert getattr(lib, s).argtypes is not None, s


def test_version_and_lengths_without_device():
    lib = _lib.load()
    assert lib.slm_version().decode().startswith("libslm_hip")
    for n in _lib.SUPPORTED_LENGTHS:
        assert lib.slm_supported_length(n) == 1
    for n in (0, 100, 300, 8192):
        assert lib.slm_supported_length(n) == 0


def test_gather_layout_offsets_match_the_shards():
    """slm_gather_layout is the offset arithmetic of slm_plan_gather_phase /
    slm_plan_gather_stats (rank order, per-hologram slabs); host-only, so it
    runs here. It must place rank r's slab where parallel.shard_range puts
    rank r's holograms."""
    from spatial_light_modulator_module_amd import parallel

    import numpy as np
    import pytest

    for total, nranks in [(512, 8), (64, 8), (7, 3), (1, 2), (0, 2), (3, 5)]:
        counts = parallel.shard_counts(total, nranks)
        for per_item in (1, 4 * 200, 1024 * 1024):
            off = _lib.gather_layout(counts, per_item)
            assert off.shape == (nranks + 1,) and off[-1] == total * per_item
            for r in range(nranks):
                rng = parallel.shard_range(total, nranks, r)
                assert off[r] == rng.start * per_item and off[r + 1] - off[r] == len(rng) * per_item
    np.testing.assert_array_equal(_lib.gather_layout([3, 0, 2], 7), [0, 21, 21, 35])
    with pytest.raises(_lib.SlmError):
        _lib.gather_layout([2, -1], 4)
