import pathlib
import sys

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
PKG_DIR = ROOT / "2ace-mmwave-channel-estimation_amd"
for p in (ROOT, PKG_DIR, ROOT / "oracle"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def gpu():
    """Fails (never skips) when selected without a GPU: -m gpu must exercise HIP."""
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    import ace_amd  # noqa: F401  -- raises if libace.so is missing
    return torch.device("cuda:0")
