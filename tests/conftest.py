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


def pytest_report_header(config):
    """The HIP library's build id (a SHA-256 of its sources and flags) in every test log."""
    try:
        import uqdme
        from uqdme_amd import build_ext
        lib = uqdme.load_library()
        got = lib.uq_build_id().decode()
        return [f"uqdme library build id: {got} ({'matches' if got == build_ext.build_id() else 'STALE vs'} sources)"]
    except Exception as e:  # noqa: BLE001  (the header must never break collection)
        return [f"uqdme library: not loaded ({e})"]


@pytest.fixture(autouse=True, scope="module")
def _release_output_pool():
    """The one-shot APIs keep output sets of large batches (outpool.py); release them after
    each test module so a later module's large allocations do not compete with them."""
    yield
    mod = sys.modules.get("uqdme_amd.outpool")
    if mod is not None:
        mod.POOL.clear()
