import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built HIP library")


@pytest.fixture(scope="session")
def gpu_ready():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no ROCm GPU is visible")
    import uqdme
    uqdme.load_library()   # fails loudly if the extension is missing
    return True
