import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); runs the HIP engine")


@pytest.fixture(scope="session")
def oracle():
    from oracle import cpu_ref

    cpu_ref.lib()
    return cpu_ref
