"""LR scheduler wrapper with automatic stepping (reference ``pytorch/_lr_scheduler.py``)."""
import enum
from typing import Any, Dict, List

import torch


class LRScheduler:
    """Wraps a ``torch.optim.lr_scheduler`` and records when the controller should step it.

    ``STEP_EVERY_EPOCH``: stepped after each training epoch (epoch = ``len(training loader)``
    batches); ``STEP_EVERY_BATCH``: after every batch; ``MANUAL_STEP``: never by the framework.
    """

    class StepMode(enum.Enum):
        STEP_EVERY_EPOCH = 1
        STEP_EVERY_BATCH = 2
        MANUAL_STEP = 3

    def __init__(self, scheduler: Any, step_mode: "LRScheduler.StepMode") -> None:
        if scheduler is None:
            raise ValueError("scheduler must not be None")
        if not isinstance(step_mode, LRScheduler.StepMode):
            raise TypeError("step_mode must be an LRScheduler.StepMode")
        self._scheduler = scheduler
        self._step_mode = step_mode

    def step(self, *args: Any, **kwargs: Any) -> None:
        self._scheduler.step(*args, **kwargs)

    def get_last_lr(self) -> List[float]:
        return self._scheduler.get_last_lr()  # type: ignore

    def load_state_dict(self, state_dict: Dict[Any, Any]) -> None:
        self._scheduler.load_state_dict(state_dict)

    def state_dict(self) -> Dict[Any, Any]:
        return self._scheduler.state_dict()  # type: ignore


# torch moved the base class name across releases; expose the one that exists
TorchLRScheduler = getattr(torch.optim.lr_scheduler, "LRScheduler", getattr(torch.optim.lr_scheduler, "_LRScheduler", object))
