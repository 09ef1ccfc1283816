"""Global average pooling (torchvision ``avgpool`` + ``flatten``)."""
from __future__ import annotations

import torch

from . import registry


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] (any memory format, any float dtype) -> [N, C] in x.dtype."""
    if registry.use_hip(x) and x.dim() == 4:
        from . import pooling_hip
        return pooling_hip.global_avg_pool(x)
    return x.float().mean(dim=(2, 3)).to(x.dtype)
