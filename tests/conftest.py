"""Test configuration: import paths and the `gpu` marker.

`-m "not gpu"` runs on any CPU host (oracle vs golden vectors, host logic,
library exports, gloo multi-process tests); `-m gpu` runs the parity tests
through the C ABI on an MI355X.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "hm-retrieval-two-tower_amd")
for p in (ROOT, PKG_DIR, os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)

import pytest  # noqa: E402


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libtt.so on cuda:0)")


@pytest.fixture(autouse=True)
def _segv_backtrace():
    """TT_SEGV_BT=<file> (diagnostic): a native backtrace of a host crash
    appended to <file> (tools/segv_bt.c), installed ahead of faulthandler at
    every test."""
    if os.environ.get("TT_SEGV_BT"):
        import ctypes
        import gc

        import torch

        graphs = sum(1 for o in gc.get_objects() if isinstance(o, torch.cuda.CUDAGraph))
        with open(os.environ["TT_SEGV_BT"], "a") as f:
            f.write(f"[segv_bt] test start: {graphs} live CUDAGraph objects\n")
        ctypes.CDLL(os.path.join(ROOT, "tools", "pbin", "libsegv_bt.so")).tt_segv_bt_install(os.environ["TT_SEGV_BT"].encode())
    yield


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but torch.cuda.is_available() is False")
    return torch.device("cuda:0")
