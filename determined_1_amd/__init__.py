"""determined_1_amd: an MI355X-native (gfx950 / CDNA4) deep-learning training platform with the
capabilities, Trial API, experiment-config schema and checkpoint format of Determined
(reference: stoksc/determined-1 @ 0.13.10.dev0).

Layout:
  ops/        hand-written HIP kernels (fused optimizers, grad norm / AMP, cast, input pipeline)
              and the flat parameter/gradient arenas built on them
  parallel/   RCCL/xGMI data parallelism: process groups, bucketed overlapped all-reduce, launcher
  pytorch/    the PyTorchTrial API (context, controller, data, reducers, LR schedulers, callbacks)
  models/     model zoo (ResNet, CIFAR/MNIST CNNs, BERT-style encoder, test fixtures)
  harness/    the trial-process layers (master socket, workload manager, rank fan-out, entrypoints)
  config/     experiment-config schema, defaults, validation, Length
  storage/    checkpoint storage managers (shared_fs, s3, gcs, hdfs)
  searcher/   Python bindings of the native C++ hyperparameter searchers (native/)
  experimental/ native API and local/test-mode execution
  tensorboard/  tfevents writer + metric writer callbacks
  cli/, sdk/  ``det`` command line and Python SDK
"""
from determined_1_amd._version import __version__
from determined_1_amd import errors
from determined_1_amd.config import ExperimentConfig
from determined_1_amd.env import EnvContext, RendezvousInfo
from determined_1_amd.errors import InvalidHP
from determined_1_amd.parallel.dist import DistributedConfig, RankInfo
from determined_1_amd.trial import (
    CallbackTrialController,
    DistributedContext,
    LoopTrialController,
    NativeContext,
    Trial,
    TrialContext,
    TrialController,
)
from determined_1_amd.workload import Workload

# reference name of the distributed config object
HorovodContext = DistributedConfig

__all__ = [
    "CallbackTrialController",
    "DistributedConfig",
    "DistributedContext",
    "EnvContext",
    "ExperimentConfig",
    "HorovodContext",
    "InvalidHP",
    "LoopTrialController",
    "NativeContext",
    "RankInfo",
    "RendezvousInfo",
    "Trial",
    "TrialContext",
    "TrialController",
    "Workload",
    "__version__",
    "errors",
]
