import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (str(ROOT), str(ROOT / "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")


@pytest.fixture(scope="session")
def ctx():
    import torch
    import vortex_amd as V
    assert torch.cuda.is_available(), "gpu tests need a GPU"
    c = V.Context(0)
    yield c
    c.close()


@pytest.fixture(scope="session")
def lineitem_file_bytes():
    """BASELINE C5's whole file (92 chunks x 16 columns, bench.c5_file), written once per
    session and shared by the tests that read it."""
    import bench
    return bench.c5_file(None, 0)
