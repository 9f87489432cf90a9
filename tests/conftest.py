import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running test")
    config.addinivalue_line("markers", "reference: compares against the read-only reference tree")


@pytest.fixture(scope="session")
def reference_core():
    """Import the reference RAFT read-only (skips where the tree is absent, e.g. on the GPU box)."""
    if not os.path.isdir(os.path.join(REFERENCE, "core")):
        pytest.skip("reference tree not available")
    os.environ.setdefault("PYTHONDONTWRITEBYTECODE", "1")
    sys.dont_write_bytecode = True
    if REFERENCE not in sys.path:
        sys.path.append(REFERENCE)
    import importlib

    return importlib.import_module("core.raft")


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from raft_ros_amd.ops import _ext

    assert _ext.is_loaded(), f"native extension must load on the GPU box: {_ext.load_error()}"
    return torch.device("cuda", 0)
