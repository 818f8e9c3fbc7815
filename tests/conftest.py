import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: longer-running CPU test")
    # Build the native core in-tree once per session (incremental).
    from flex_gpu_scheduler_amd import build_ext

    build_ext.build_core(verbose=False)


@pytest.fixture
def store():
    from flex_gpu_scheduler_amd import Store

    return Store()
