"""Native API, local/test execution and the Python SDK (``determined.experimental`` equivalent)."""
from determined_1_amd.experimental._local import (
    load_model_def,
    make_controller,
    make_local_env,
    make_test_workloads,
    run_local_test,
    sample_hparams,
    test_one_batch,
)
from determined_1_amd.experimental.native import create
from determined_1_amd.experimental.client import (
    Checkpoint,
    Determined,
    ExperimentReference,
    Model,
    ModelOrderBy,
    ModelSortBy,
    TrialReference,
    load_checkpoint,
)

__all__ = [
    "Checkpoint",
    "Determined",
    "create",
    "ExperimentReference",
    "TrialReference",
    "load_checkpoint",
    "Model",
    "ModelOrderBy",
    "ModelSortBy",
    "load_model_def",
    "make_controller",
    "make_local_env",
    "make_test_workloads",
    "run_local_test",
    "sample_hparams",
    "test_one_batch",
]
