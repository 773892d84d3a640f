import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def native_build():
    """Build the shim + mock HIP runtime once per session (CPU-safe)."""
    from k8s_vgpu_scheduler_amd.utils import build
    build.build_shim()
    mock_lib, driver = build.build_mock()
    return {"shim": build.SHIM_SO, "mock_lib": mock_lib, "driver": driver, "roctx": build.MOCK_ROCTX,
            "boardd": build.build_boardd(), "mock_smi": build.MOCK_SMI}
