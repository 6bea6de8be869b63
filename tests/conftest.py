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
    gpu = request.node.get_closest_marker("gpu") is not None
    if gpu:
        import torch
        cur = torch.cuda.current_stream()
        if cur != torch.cuda.default_stream():
            # a test must not inherit a switched current stream: work it enqueues would not be
            # ordered with the default stream's (and threads' pool streams sync only with that)
            pytest.fail(f"test started on a non-default current stream {cur} (leaked by an earlier test)")
    yield
    if gpu:
        gc.collect()
