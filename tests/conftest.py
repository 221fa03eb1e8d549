import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def core():
    from shellac_amd._native import core as _core

    return _core()


@pytest.fixture
def cuda_dev():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test scheduled on a machine without a GPU")
    return torch.device("cuda", 0)
