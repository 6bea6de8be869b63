import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (native HIP kernels)")


import gc  # noqa: E402

import pytest  # noqa: E402


@pytest.fixture(autouse=True)
def _collect_gpu_garbage(request):
    """GPU tests drop models that hold captured graphs, streams and communicators; collect them
    right after the test instead of at an arbitrary later point (inside another test's capture)."""
    yield
    if request.node.get_closest_marker("gpu") is not None:
        gc.collect()
