"""Distributed-training configuration and process-group bootstrap (replaces the reference's
Horovod glue, ``harness/determined/horovod.py:166-254`` and its ZMQ control plane
``harness/determined/ipc.py``).

MI355X design:
  * one process per GPU; ``torch.distributed`` with backend ``"nccl"`` == RCCL over xGMI for
    tensors (gradient buckets, parameter/optimizer-state broadcast);
  * a second, CPU-side ``gloo`` group is the *control plane* (metric gathers to the chief,
    object broadcast, barriers) so small pickled messages never queue behind gradient traffic on
    the RCCL stream and never touch HBM;
  * rendezvous is torch's native C++ TCPStore on the chief's address (rank 0), replacing the
    reference's SSH + ``horovodrun`` launch and ZMQ sockets.
"""
import datetime
import logging
import os
import pickle
from typing import Any, Dict, List, Optional

import torch
import torch.distributed as dist

from determined_1_amd import constants


class DistributedConfig:
    """What the reference calls ``HorovodContext``: whether multi-process DP is on and its knobs.

    ``use = multi_machine or (multi_slot and not native_parallel)`` (reference horovod.py:196-200).
    """

    def __init__(
        self,
        use: bool,
        aggregation_frequency: int = 1,
        average_aggregated_gradients: bool = True,
        average_training_metrics: bool = False,
        grad_compression: bool = False,
        fusion_threshold_mb: int = 64,
        cycle_time_ms: int = 5,
        auto_tune: bool = False,
        compression_dtype: str = "bfloat16",
        grad_reduction: str = "fp32_accum",
        rccl: Optional[Dict[str, Any]] = None,
    ) -> None:
        self.use = use
        self.aggregation_frequency = max(1, int(aggregation_frequency))
        self.average_aggregated_gradients = average_aggregated_gradients
        self.average_training_metrics = average_training_metrics
        self.grad_compression = grad_compression
        self.fusion_threshold_mb = fusion_threshold_mb
        self.cycle_time_ms = cycle_time_ms
        self.auto_tune = auto_tune
        self.compression_dtype = compression_dtype
        self.grad_reduction = grad_reduction
        self.rccl = dict(rccl or {})

    # reference attribute name used by user code
    @property
    def fp16_compression(self) -> bool:
        return self.grad_compression

    @staticmethod
    def from_configs(experiment_config: Dict[str, Any], world_size: int = 1, num_agents: int = 1) -> "DistributedConfig":
        res = experiment_config.get("resources", {})
        opt = experiment_config.get("optimizations", {})
        slots = int(res.get("slots_per_trial", 1))
        native_parallel = bool(res.get("native_parallel", False))
        multi_machine = num_agents > 1
        multi_slot = slots > 1 or world_size > 1
        use = multi_machine or (multi_slot and not native_parallel)
        # DET_FORCE_DISTRIBUTED=1: run the multi-process path (process groups, bucketer,
        # broadcasts) even with one rank -- exercises RCCL on a one-GPU box.
        if os.environ.get("DET_FORCE_DISTRIBUTED", "0") == "1":
            use = True
        return DistributedConfig(
            use=use,
            aggregation_frequency=int(opt.get("aggregation_frequency", 1)),
            average_aggregated_gradients=bool(opt.get("average_aggregated_gradients", True)),
            average_training_metrics=bool(opt.get("average_training_metrics", False)),
            grad_compression=bool(opt.get("gradient_compression", False)),
            fusion_threshold_mb=int(opt.get("tensor_fusion_threshold", 64)),
            cycle_time_ms=int(opt.get("tensor_fusion_cycle_time", 5)),
            auto_tune=bool(opt.get("auto_tune_tensor_fusion", False)),
            compression_dtype=str(opt.get("gradient_compression_dtype", "bfloat16")),
            grad_reduction=str(opt.get("grad_reduction", "fp32_accum")),
            rccl=opt.get("rccl") or {},
        )

    def log_inapplicable(self) -> None:
        """``tensor_fusion_cycle_time`` is Horovod's background-thread cycle; buckets here launch the
        moment backward completes them, so a non-default value is accepted and has no effect."""
        if self.use and self.cycle_time_ms != 5:
            logging.info("optimizations.tensor_fusion_cycle_time=%s has no effect: gradient buckets are "
                         "launched as soon as backward completes them (no fusion cycle)", self.cycle_time_ms)

    @staticmethod
    def single() -> "DistributedConfig":
        return DistributedConfig(use=False)


class RankInfo:
    """Rank layout of this process, from the launcher env (RANK/LOCAL_RANK/WORLD_SIZE/...)."""

    def __init__(self, rank: int = 0, local_rank: int = 0, size: int = 1, local_size: int = 1,
                 cross_rank: int = 0, cross_size: int = 1) -> None:
        self.rank = rank
        self.local_rank = local_rank
        self.size = size
        self.local_size = local_size
        self.cross_rank = cross_rank
        self.cross_size = cross_size

    @staticmethod
    def from_env(env: Optional[Dict[str, str]] = None) -> "RankInfo":
        e = os.environ if env is None else env
        size = int(e.get("WORLD_SIZE", "1"))
        local_size = int(e.get("LOCAL_WORLD_SIZE", str(size)))
        rank = int(e.get("RANK", "0"))
        return RankInfo(
            rank=rank,
            local_rank=int(e.get("LOCAL_RANK", "0")),
            size=size,
            local_size=local_size,
            cross_rank=int(e.get("GROUP_RANK", e.get("DET_CROSS_RANK", str(rank // max(1, local_size))))),
            cross_size=int(e.get("DET_CROSS_SIZE", str(max(1, size // max(1, local_size))))),
        )

    def is_chief(self) -> bool:
        return self.rank == 0


_control_group = None  # gloo group for CPU-side control collectives


def local_cuda_device(local_rank: int) -> torch.device:
    """GPU of this rank: ``cuda:<local_rank>`` (one process per GPU).  Rehearsal mode
    ``DET_DIST_SHARE_GPU=1`` folds ranks onto the visible GPUs (``local_rank % count``) so a
    multi-rank data-parallel run (with ``DET_DIST_BACKEND=gloo``) can exercise the GPU-side
    gradient path on a one-GPU box; RCCL itself refuses two ranks on one device."""
    if os.environ.get("DET_DIST_SHARE_GPU", "0") == "1":
        return torch.device("cuda", local_rank % max(1, torch.cuda.device_count()))
    return torch.device("cuda", local_rank)


def is_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def init_process_groups(device: torch.device, timeout_s: int = constants.DIST_STARTUP_TIMEOUT_SECONDS) -> None:
    """Create the RCCL (or gloo on CPU) data group and the gloo control group from env://."""
    global _control_group
    if is_initialized():
        if _control_group is None:
            _control_group = dist.new_group(backend="gloo")
        return
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    backend = "nccl" if device.type == "cuda" else "gloo"
    backend = os.environ.get("DET_DIST_BACKEND", backend)  # gloo: GPU-sharing rehearsals (see above)
    kwargs = {}
    if backend == "nccl":
        kwargs["device_id"] = device  # eager RCCL communicator init, bound to this GPU
        # fresh events per collective instead of torch's event cache: a cached event re-recorded by a
        # collective inside a hipGraph capture can still be queried by the watchdog thread for the
        # eager work that last used it ("operation not permitted on an event last recorded in a
        # capturing stream", seen once in the world-1 DP graph test, profiles/r6_s76_final_rehearsal.txt)
        os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")
    dist.init_process_group(backend=backend, timeout=datetime.timedelta(seconds=timeout_s), **kwargs)
    _control_group = dist.new_group(backend="gloo") if backend == "nccl" else dist.group.WORLD
    logging.info("initialized %s data group + gloo control group: rank %d/%d", backend, dist.get_rank(),
                 dist.get_world_size())


def control_group() -> Any:
    return _control_group


def shutdown() -> None:
    global _control_group
    if is_initialized():
        dist.destroy_process_group()
    _control_group = None


# ----------------------------------------------------------------------------------------------
# control-plane collectives over gloo (replace ZMQ gather/broadcast/barrier, SURVEY C-4..C-6)
# ----------------------------------------------------------------------------------------------
def barrier() -> None:
    if is_initialized():
        dist.barrier(group=_control_group)


def broadcast_object(obj: Any, src: int = 0) -> Any:
    if not is_initialized():
        return obj
    lst = [obj]
    dist.broadcast_object_list(lst, src=src, group=_control_group)
    return lst[0]


def gather_to_chief(obj: Any) -> Optional[List[Any]]:
    """Gather one picklable object per rank to rank 0 (returns the list on rank 0, else None)."""
    if not is_initialized():
        return [obj]
    rank = dist.get_rank()
    out = [None] * dist.get_world_size() if rank == 0 else None
    dist.gather_object(obj, out, dst=0, group=_control_group)
    return out


def allgather_object(obj: Any) -> List[Any]:
    if not is_initialized():
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj, group=_control_group)
    return out


def pickled_size(obj: Any) -> int:
    return len(pickle.dumps(obj))
