"""Global average pooling (torchvision ``avgpool`` + ``flatten``) and the ImageNet
stem's MaxPool2d(3, 2, 1), on the HIP kernels when the input is a bf16 NHWC GPU
tensor."""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import registry


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """[N, C, H, W] (any memory format, any float dtype) -> [N, C] in x.dtype."""
    if registry.use_hip(x) and x.dim() == 4:
        from . import pooling_hip
        return pooling_hip.global_avg_pool(x)
    return (x if x.dtype == torch.float64 else x.float()).mean(dim=(2, 3)).to(x.dtype)


class MaxPool2d(nn.Module):
    """``nn.MaxPool2d`` drop-in (no parameters, same state-dict keys): the HIP kernel records
    each window's argmax so the backward is a deterministic gather (csrc/eval.hip)."""

    def __init__(self, kernel_size: int = 3, stride: int = 2, padding: int = 1):
        super().__init__()
        self.kernel_size, self.stride, self.padding = kernel_size, stride, padding

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if (registry.use_hip(x) and x.dim() == 4 and x.dtype == torch.bfloat16
                and x.shape[1] % 8 == 0):
            from . import pooling_hip
            return pooling_hip.MaxPoolHipFn.apply(x, self.kernel_size, self.stride, self.padding)
        return F.max_pool2d(x, self.kernel_size, self.stride, self.padding)

    def extra_repr(self) -> str:
        return f"kernel_size={self.kernel_size}, stride={self.stride}, padding={self.padding}"
