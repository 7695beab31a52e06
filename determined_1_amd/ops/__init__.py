"""Hand-written gfx950 (MI355X / CDNA4) kernels and the flat-arena machinery built on them."""
from determined_1_amd.ops._lib import KernelLibraryMissing, get_lib, lib_available
from determined_1_amd.ops.arena import Arena, build_arenas
from determined_1_amd.ops.functional import (
    MultiTensorCopy,
    NormWorkspace,
    global_norm_,
    scale_cast_,
    u8_normalize,
    unscale_check_,
)
from determined_1_amd.ops.optim import FusedOptimizer, fused_kind

__all__ = [
    "Arena",
    "FusedOptimizer",
    "KernelLibraryMissing",
    "MultiTensorCopy",
    "NormWorkspace",
    "build_arenas",
    "fused_kind",
    "get_lib",
    "global_norm_",
    "lib_available",
    "scale_cast_",
    "u8_normalize",
    "unscale_check_",
]
