import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


@pytest.hookimpl(tryfirst=True)
def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running test")
    # The CPU suite (``-m "not gpu"``) runs on pytest-xdist workers: 13.7 min serially, ~7 min on 4-6
    # workers (every test uses its own ports / tmp dirs).  GPU runs stay in one process (one test
    # process per GPU box).  DET_TEST_WORKERS=0 runs serially; an explicit ``-n`` wins.
    workers = int(os.environ.get("DET_TEST_WORKERS", "4"))
    if (workers > 0 and config.pluginmanager.hasplugin("xdist") and getattr(config.option, "numprocesses", None) is None
            and (getattr(config.option, "markexpr", "") or "").replace(" ", "") == "notgpu"
            and not os.environ.get("PYTEST_XDIST_WORKER")):
        # what xdist's own pytest_cmdline_main derives from ``-n`` (it has run by now)
        config.option.numprocesses = workers
        if getattr(config.option, "dist", "no") == "no":
            config.option.dist = "load"
        config.option.tx = ["popen"] * workers


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

