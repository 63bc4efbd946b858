import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) device")


def _gpu_present() -> bool:
    try:
        from volsync_amd import _lib
        return _lib.device_count() > 0
    except ImportError:
        return False


@pytest.fixture(scope="session")
def gpu():
    """Fails (not skips) when a gpu-marked test runs without a device: the GPU
    suite must never pass on a silent fallback."""
    if not _gpu_present():
        pytest.fail("gpu test requested but no HIP device / libvsgpu.so available")
    import torch
    return torch.device("cuda:0")
