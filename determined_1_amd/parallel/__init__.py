"""Data-parallel training over RCCL/xGMI: process groups, bucketed gradient all-reduce, launcher."""
from determined_1_amd.parallel.dist import (
    DistributedConfig,
    RankInfo,
    allgather_object,
    barrier,
    broadcast_object,
    gather_to_chief,
    init_process_groups,
    is_initialized,
)
from determined_1_amd.parallel.ddp import GradientBucketer, broadcast_arenas, broadcast_tensors_coalesced

__all__ = [
    "DistributedConfig",
    "GradientBucketer",
    "RankInfo",
    "allgather_object",
    "barrier",
    "broadcast_arenas",
    "broadcast_object",
    "broadcast_tensors_coalesced",
    "gather_to_chief",
    "init_process_groups",
    "is_initialized",
]
