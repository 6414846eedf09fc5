import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# run-time compiled kernels: a test session has its own on-disk code-object
# cache, so tests that count compiles do not depend on earlier runs
if "RSAMD_JIT_CACHE_DIR" not in os.environ:
    import tempfile

    os.environ["RSAMD_JIT_CACHE_DIR"] = tempfile.mkdtemp(prefix="rsamd_jit_")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C ABI)")


def _has_gpu() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(autouse=True)
def _gpu_required(request):
    # A gpu-marked test must run on a GPU: it fails (never skips) without one,
    # so a green `-m gpu` run always means the HIP path executed.
    if request.node.get_closest_marker("gpu") and not _has_gpu():
        pytest.fail("gpu test needs a visible HIP device")


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def rslib():
    import reedsolomon_amd
    from reedsolomon_amd import build

    build.build()
    return reedsolomon_amd
