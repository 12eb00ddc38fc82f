import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


@pytest.fixture(scope="session")
def lib():
    from fantoch_amd import _lib
    return _lib.load()


@pytest.fixture(scope="session")
def gpu(lib):
    if lib.fx_device_count() <= 0:
        pytest.fail("GPU test on a machine without a GPU: the HIP path has no fallback")
    return lib
