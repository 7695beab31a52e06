"""PyTorch Trial API (``determined.pytorch`` equivalent)."""
from determined_1_amd.pytorch._callback import ClipGradsL2Norm, ClipGradsL2Value, PyTorchCallback
from determined_1_amd.pytorch._data import (
    BatchChunk,
    ChunkedBatches,
    ChunkPrefetcher,
    DataLoader,
    DevicePrefetcher,
    DistributedBatchSampler,
    RepeatBatchSampler,
    SkipBatchSampler,
    TorchData,
    _Data,
    adapt_batch_sampler,
    data_length,
    passthrough_collate,
    to_device,
)
from determined_1_amd.pytorch._lr_scheduler import LRScheduler
from determined_1_amd.pytorch._reducer import Reducer, _reduce_metrics
from determined_1_amd.pytorch._context import ClipGradsNorm, PyTorchTrialContext
from determined_1_amd.pytorch._trial import PyTorchTrial, PyTorchTrialController, reset_parameters

__all__ = [
    "ClipGradsL2Norm",
    "ClipGradsL2Value",
    "ClipGradsNorm",
    "DataLoader",
    "DevicePrefetcher",
    "BatchChunk",
    "ChunkedBatches",
    "ChunkPrefetcher",
    "passthrough_collate",
    "DistributedBatchSampler",
    "LRScheduler",
    "PyTorchCallback",
    "PyTorchTrial",
    "PyTorchTrialContext",
    "PyTorchTrialController",
    "Reducer",
    "RepeatBatchSampler",
    "SkipBatchSampler",
    "TorchData",
    "adapt_batch_sampler",
    "data_length",
    "reset_parameters",
    "to_device",
]
