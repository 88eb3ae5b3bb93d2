"""pytest configuration: the ``gpu`` marker and the in-tree native build.

CPU tests (``-m "not gpu"``) run everywhere (gloo for multi-process); GPU tests need a real MI355X
and the gfx950 extension ``distriflow_amd/_C.so``, which is (re)built here once per session.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session", autouse=True)
def _native_build():
    from distriflow_amd import _build

    _build.build()
    yield


def gpu_available():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False
