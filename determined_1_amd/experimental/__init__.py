"""Native API and local/test execution (``determined.experimental`` equivalent)."""
from determined_1_amd.experimental._local import (
    make_controller,
    make_local_env,
    make_test_workloads,
    sample_hparams,
    test_one_batch,
)

__all__ = ["make_controller", "make_local_env", "make_test_workloads", "sample_hparams", "test_one_batch"]
