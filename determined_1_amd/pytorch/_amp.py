"""Native mixed precision that honours the reference's ``configure_apex_amp`` API.

Reference: ``harness/determined/pytorch/_pytorch_context.py:262-382`` (apex.amp.initialize
O0-O3, dynamic loss scale up to 2**24, ``amp_state`` in checkpoints ``_pytorch_trial.py:664-675``).

MI355X mapping (no apex on ROCm, and bf16 is the native fast type of CDNA4 MFMA):
  * ``O0``  fp32, nothing to do.
  * ``O1``  ``torch.autocast`` around forward/eval; dtype **bf16 by default** (fp32 exponent range,
            so no loss scaling is needed); ``cast_model_type=torch.float16`` (or
            ``DET_AMP_DTYPE=float16``) selects fp16 with a dynamic loss scaler.
  * ``O2``  model weights cast to bf16/fp16 (BatchNorm kept fp32 unless
            ``keep_batchnorm_fp32=False``); the fused optimizer keeps fp32 *master* weights in its
            arena and writes the low-precision copy back in the same kernel (``det_*_step``
            ``out_model``); floating inputs are cast by a forward pre-hook.
  * ``O3``  like O2 with BatchNorm cast too.

Dynamic loss scaling never syncs the host: overflow is a device flag (``found_inf``) produced by
the gradient-norm / unscale kernels, consumed by the optimizer kernel (skip step) and by
``torch._amp_update_scale_`` (scale backoff / growth).
"""
import os
from typing import Any, Dict, Optional

import torch

OPT_LEVELS = ("O0", "O1", "O2", "O3")


def _env_dtype() -> Optional[torch.dtype]:
    v = os.environ.get("DET_AMP_DTYPE", "").lower()
    if v in ("float16", "fp16", "half"):
        return torch.float16
    if v in ("bfloat16", "bf16"):
        return torch.bfloat16
    return None


class DynamicLossScaler:
    """Device-resident loss scale with apex-compatible ``state_dict``."""

    def __init__(self, device: torch.device, init_scale: float = 2.0 ** 16, growth_factor: float = 2.0,
                 backoff_factor: float = 0.5, growth_interval: int = 2000, max_scale: float = 2.0 ** 24,
                 min_scale: Optional[float] = None, dynamic: bool = True) -> None:
        self.device = device
        self.dynamic = dynamic
        self.growth_factor = growth_factor
        self.backoff_factor = backoff_factor
        self.growth_interval = growth_interval
        self.max_scale = max_scale
        self.min_scale = min_scale
        self.scale = torch.full((1,), min(init_scale, max_scale), dtype=torch.float32, device=device)
        self.inv_scale = torch.reciprocal(self.scale)
        self.growth_tracker = torch.zeros((1,), dtype=torch.int32, device=device)
        self.found_inf = torch.zeros((1,), dtype=torch.int32, device=device)

    def scale_loss(self, loss: torch.Tensor) -> torch.Tensor:
        return loss.float() * self.scale

    def reset_found_inf(self) -> None:
        self.found_inf.zero_()

    def update(self) -> None:
        if not self.dynamic:
            return
        torch._amp_update_scale_(
            self.scale, self.growth_tracker, self.found_inf.float(), self.growth_factor, self.backoff_factor,
            self.growth_interval,
        )
        if self.max_scale is not None or self.min_scale is not None:
            self.scale.clamp_(min=self.min_scale or 0.0, max=self.max_scale or float("inf"))
        torch.reciprocal(self.scale, out=self.inv_scale)

    def state_dict(self) -> Dict[str, Any]:
        return {"loss_scaler0": {"loss_scale": float(self.scale.item()), "unskipped": int(self.growth_tracker.item())}}

    def load_state_dict(self, sd: Dict[str, Any]) -> None:
        s = sd.get("loss_scaler0", sd)
        self.scale.fill_(float(s.get("loss_scale", self.scale.item())))
        self.growth_tracker.fill_(int(s.get("unskipped", 0)))
        torch.reciprocal(self.scale, out=self.inv_scale)


class AmpConfig:
    def __init__(self, opt_level: str, dtype: torch.dtype, keep_batchnorm_fp32: bool, scaler: Optional[DynamicLossScaler]) -> None:
        self.opt_level = opt_level
        self.dtype = dtype
        self.keep_batchnorm_fp32 = keep_batchnorm_fp32
        self.scaler = scaler

    @property
    def autocast(self) -> bool:
        return self.opt_level == "O1"

    @property
    def casts_model(self) -> bool:
        return self.opt_level in ("O2", "O3")

    def state_dict(self) -> Dict[str, Any]:
        if self.scaler is not None:
            return self.scaler.state_dict()
        return {"loss_scaler0": {"loss_scale": 1.0, "unskipped": 0}}

    def load_state_dict(self, sd: Dict[str, Any]) -> None:
        if self.scaler is not None:
            self.scaler.load_state_dict(sd)


def make_amp_config(device: torch.device, opt_level: str, cast_model_type: Optional[torch.dtype],
                    keep_batchnorm_fp32: Optional[Any], loss_scale: Optional[Any],
                    min_loss_scale: Optional[float], max_loss_scale: Optional[float]) -> AmpConfig:
    if opt_level not in OPT_LEVELS:
        raise ValueError(f"opt_level must be one of {OPT_LEVELS}, got {opt_level!r}")
    dtype = cast_model_type if cast_model_type in (torch.float16, torch.bfloat16) else (_env_dtype() or torch.bfloat16)
    if isinstance(keep_batchnorm_fp32, str):
        keep_batchnorm_fp32 = keep_batchnorm_fp32 == "True"
    keep_bn = True if keep_batchnorm_fp32 is None else bool(keep_batchnorm_fp32)
    if opt_level == "O3" and keep_batchnorm_fp32 is None:
        keep_bn = False
    scaler = None
    dynamic = loss_scale in (None, "dynamic")
    if opt_level != "O0" and (dtype == torch.float16 or loss_scale not in (None, "dynamic", 1, 1.0, "1.0")):
        init = 2.0 ** 16 if dynamic else float(loss_scale)
        scaler = DynamicLossScaler(device, init_scale=init, dynamic=dynamic and dtype == torch.float16,
                                   max_scale=max_loss_scale if max_loss_scale is not None else 2.0 ** 24,
                                   min_scale=min_loss_scale)
    return AmpConfig(opt_level, dtype, keep_bn, scaler)


# apex O2 keeps only BatchNorm in fp32 (F.batch_norm accepts a bf16 input with fp32 affine
# params); LayerNorm/GroupNorm require matching dtypes, so they are cast with the rest.
_BN_TYPES = (torch.nn.modules.batchnorm._BatchNorm,)


def cast_model(model: torch.nn.Module, dtype: torch.dtype, keep_batchnorm_fp32: bool) -> torch.nn.Module:
    """apex O2/O3 model cast: everything to ``dtype`` except normalisation layers (if kept)."""
    for m in model.modules():
        if keep_batchnorm_fp32 and isinstance(m, _BN_TYPES):
            continue
        for name, p in list(m.named_parameters(recurse=False)):
            if p.is_floating_point():
                p.data = p.data.to(dtype)
        for name, b in list(m.named_buffers(recurse=False)):
            if b is not None and b.is_floating_point():
                setattr(m, name, b.to(dtype))
    return model


def _cast_inputs_hook(dtype: torch.dtype) -> Any:
    def _cast(x: Any) -> Any:
        if isinstance(x, torch.Tensor) and x.is_floating_point() and x.dtype != dtype:
            return x.to(dtype)
        if isinstance(x, (list, tuple)):
            return type(x)(_cast(v) for v in x)
        if isinstance(x, dict):
            return {k: _cast(v) for k, v in x.items()}
        return x

    def hook(_module: torch.nn.Module, args: Any, kwargs: Any) -> Any:
        return _cast(args), _cast(kwargs)

    return hook


def install_input_cast(model: torch.nn.Module, dtype: torch.dtype) -> Any:
    return model.register_forward_pre_hook(_cast_inputs_hook(dtype), with_kwargs=True)
