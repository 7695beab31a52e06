import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from determined_1_amd.ops import build

    build.build()
    from determined_1_amd.ops import _lib

    _lib.get_lib()  # must load: GPU tests never run on an eager fallback
    return torch.device("cuda", 0)


@pytest.fixture(autouse=True)
def _freeze_earlier_objects(request):
    """CPU runs (``-m "not gpu"``): objects that outlived earlier tests (module caches, models held by
    fixtures) are moved out of the cyclic collector's view before each test.  In one long pytest
    process every gen-2 collection otherwise rescans all of them, and tests that allocate many small
    objects late in the suite ran 2-8x slower than alone (the COCO instance-load test 36 s vs 5 s).
    Not on GPU runs, where a frozen cycle could keep device memory alive for the rest of the suite."""
    if (request.config.option.markexpr or "").replace(" ", "") == "notgpu":
        import gc

        gc.freeze()
    yield
