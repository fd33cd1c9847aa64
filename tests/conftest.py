import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the product library and the oracle in-tree once per session."""
    from izpi_amd import build
    from oracle import oracle
    build.build_gpu(verbose=False)
    oracle.build()
    yield


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not gpu_available():
        pytest.skip("no HIP device")
    return 0
