"""Every official example's local test mode on the MI355X (the CPU suite runs the same configs on
the host): the trials' GPU paths — fused kernels, arenas, AMP casts — on the shrunken models."""
import pytest
import torch

from tests.test_examples import CONFIGS, test_example_local_test_mode as _run_example

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("example", sorted({p.parent for p in CONFIGS}), ids=lambda p: p.name)
def test_example_local_test_mode_on_gpu(gpu, example):
    assert torch.cuda.is_available()
    _run_example(example)
