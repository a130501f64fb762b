"""Shared fixtures.  `-m gpu` tests need an MI355X; everything else runs on CPU."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def rt():
    import go_raytracer_amd
    return go_raytracer_amd


@pytest.fixture(scope="session")
def oracle():
    from oracle import pyoracle
    pyoracle.lib()
    return pyoracle


@pytest.fixture
def tune(rt):
    """Set tuning knobs for one test (rt_tune_set); every knob is cleared afterwards."""
    rt.untune()
    yield rt.tune
    rt.untune()


@pytest.fixture(scope="session")
def gpu(rt):
    n = rt.device_count()
    if n <= 0:
        pytest.fail("gpu test run without a visible HIP device")
    return 0
