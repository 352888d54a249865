import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device and the native extension")
    config.addinivalue_line("markers", "slow: long-running test")


def _has_gpu():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU available")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


def devices():
    """Parametrisation helper: cpu always, cuda as a gpu-marked case."""
    return [pytest.param("cpu"), pytest.param("cuda", marks=pytest.mark.gpu)]


@pytest.fixture(autouse=True)
def _restore_bh_config():
    """Tests switch paths with ``beforeholiday_amd.config.set(...)``; every test starts from and leaves
    behind the process's configuration as it was."""
    import dataclasses

    from beforeholiday_amd import config

    old = config.get()
    yield
    if config.get() != old:
        config.set(**dataclasses.asdict(old))
