"""Shared pytest configuration.

The HIP library is loaded before anything imports torch so that one HIP
runtime (the system ROCm one libslm_hip.so links) serves the whole process.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import spatial_light_modulator_module_amd  # noqa: E402,F401  (loads libslm_hip.so first)

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
