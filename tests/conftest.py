import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")


@pytest.fixture(scope="session")
def has_gpu():
    from chubaofs_amd import _lib
    return _lib.device_count() > 0


@pytest.fixture(autouse=True)
def _skip_gpu_without_device(request):
    if request.node.get_closest_marker("gpu"):
        from chubaofs_amd import _lib
        if _lib.device_count() == 0:
            pytest.fail("gpu test selected but no HIP device is visible")
