"""Dense layer dispatch (projection head / classifier GEMMs)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from . import registry
from .conv import effective_weight


def linear_module(mod, x: torch.Tensor) -> torch.Tensor:
    """Forward of ``models.heads.Linear``: bf16 GPU activations run the MFMA GEMM kernels,
    everything else (fp32 probes, CPU) runs ``F.linear``."""
    if x.dtype == torch.bfloat16 and registry.use_hip(x):
        from . import gemm_hip
        out = gemm_hip.linear(x, None, None, weight_param=mod.weight, bias_param=mod.bias,
                              emit_stats=getattr(mod, "emit_bn_stats", False) and mod.training)
        if out is not None:
            return out
    w = effective_weight(mod)
    if w.dtype != x.dtype:
        w = w.to(x.dtype)
    b = mod.bias
    if b is not None and b.dtype != x.dtype:
        b = b.to(x.dtype)
    return F.linear(x, w, b)
