import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT / "trex-emu_amd", ROOT / "oracle", ROOT / "tests"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running (full BASELINE sizes)")


@pytest.fixture(scope="session")
def oracle_built():
    import pyoracle
    pyoracle.build()
    return pyoracle


@pytest.fixture(scope="session")
def lib():
    """libemurx.so loaded (built first if missing); loading touches no GPU."""
    from emurx import abi
    if not abi.LIB_PATH.exists():
        import subprocess
        subprocess.run(["make", "-s", "-C", str(abi.PKG_ROOT)], check=True)
    return abi.load()


@pytest.fixture(scope="session")
def gpu_ok():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    return torch
