"""The seed gradient of scalar losses as one shared constant tensor per (dtype, device).

``PyTorchTrialContext.backward`` passes it to ``loss.backward`` instead of letting autograd build
``ones_like(loss)`` (a fill launch per backward), and a loss op whose forward can also produce its
gradient for a seed of exactly 1 hands that over without a launch when its backward receives this
tensor (``ops.cnn._XEnt``).  Created outside hipGraph captures only: a tensor allocated inside one
takes an address the graph reuses for earlier temporaries, which a replay would overwrite.
"""
from typing import Dict, Optional, Tuple

import torch

_UNIT = {}  # type: Dict[Tuple[torch.dtype, torch.device], torch.Tensor]
_PTRS = set()  # data pointers of the cached unit tensors


def unit_for(loss: torch.Tensor) -> Optional[torch.Tensor]:
    """The shared unit seed for ``loss`` (a scalar GPU tensor with a grad_fn), or None."""
    if loss.dim() != 0 or not loss.is_cuda or loss.grad_fn is None:
        return None  # (a leaf loss would keep the seed as its .grad and accumulate into it)
    key = (loss.dtype, loss.device)
    t = _UNIT.get(key)
    if t is None:
        if torch.cuda.is_current_stream_capturing():
            return None
        t = _UNIT[key] = torch.ones((), dtype=loss.dtype, device=loss.device)
        _PTRS.add(t.data_ptr())
    return t


def is_unit(g: torch.Tensor) -> bool:
    """True when ``g`` is (a view of) a shared unit seed: its value is 1 without reading it."""
    return g.is_cuda and g.numel() == 1 and g.data_ptr() in _PTRS
