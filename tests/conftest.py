import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

SCENES = ROOT / "tests" / "scenes"
GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the native library and the oracle in-tree if they are missing (no-op when fresh)."""
    from cuda_pathtracer_amd import build as B
    B.build_all()
    yield


@pytest.fixture(scope="session")
def cornell_path() -> str:
    return str(SCENES / "cornell.json")


@pytest.fixture(scope="session")
def gpu_device():
    import torch
    assert torch.cuda.is_available(), "GPU test run without a visible GPU"
    torch.cuda.set_device(0)
    return torch.device("cuda", 0)
