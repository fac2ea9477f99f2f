"""Shared pytest configuration. The package imports no torch; libslm_hip.so is
loaded here so that a missing build fails the session at once."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from spatial_light_modulator_module_amd import _lib as _slm_lib  # noqa: E402

_slm_lib.load()

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run on the MI355X box)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def gpu():
    from spatial_light_modulator_module_amd import _lib

    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible: gpu-marked tests must run on the MI355X box")
    _lib.init()
    return _lib
