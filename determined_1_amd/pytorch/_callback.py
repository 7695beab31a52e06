"""PyTorchTrial callbacks (reference ``pytorch/_callback.py``)."""
from typing import Any, Dict, Iterator

import torch


class PyTorchCallback:
    """Hooks invoked by the PyTorch trial controller.  ``state_dict``/``load_state_dict`` are
    saved in and restored from checkpoints (under ``callbacks``)."""

    def on_before_optimizer_step(self, parameters: Iterator) -> None:
        """Deprecated: only called by the legacy build_model()/optimizer() interface."""

    def on_validation_start(self) -> None:
        pass

    def on_validation_end(self, metrics: Dict[str, Any]) -> None:
        pass

    def on_validation_step_start(self) -> None:
        """Deprecated alias of on_validation_start."""

    def on_validation_step_end(self, metrics: Dict[str, Any]) -> None:
        """Deprecated alias of on_validation_end."""

    def on_checkpoint_end(self, checkpoint_dir: str) -> None:
        pass

    def on_train_step_start(self, step_id: int) -> None:
        pass

    def on_train_step_end(self, step_id: int, metrics: Dict[str, Any]) -> None:
        pass

    def state_dict(self) -> Dict[str, Any]:
        return {}

    def load_state_dict(self, state_dict: Dict[str, Any]) -> None:
        pass


class ClipGradsL2Norm(PyTorchCallback):
    """Deprecated callback: clip gradients to an L2 norm before the optimizer step."""

    def __init__(self, clip_value: float) -> None:
        self._clip_value = clip_value

    def on_before_optimizer_step(self, parameters: Iterator) -> None:
        torch.nn.utils.clip_grad_norm_(parameters, self._clip_value)  # type: ignore


class ClipGradsL2Value(PyTorchCallback):
    """Deprecated callback: clip gradient values before the optimizer step."""

    def __init__(self, clip_value: float) -> None:
        self._clip_value = clip_value

    def on_before_optimizer_step(self, parameters: Iterator) -> None:
        torch.nn.utils.clip_grad_value_(parameters, self._clip_value)  # type: ignore
