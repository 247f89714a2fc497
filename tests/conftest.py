import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs a real MI355X (HIP device + built flexflow_amd._C)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def ffC():
    """The compiled HIP kernel module; GPU tests fail loudly (not skip) if it is missing."""
    import torch  # noqa: F401
    from flexflow_amd import _C
    return _C
