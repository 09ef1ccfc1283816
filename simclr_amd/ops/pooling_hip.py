"""Global average pool (avgpool + flatten, ``csrc/misc.hip``) and max pool with argmax
(``csrc/eval.hip``) as autograd functions on bf16 NHWC tensors."""
from __future__ import annotations

import torch

from . import _ext
from .conv_hip import _nhwc


class AvgPoolHipFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ops = _ext.ops()
        N, C, H, W = x.shape
        y = torch.empty((N, C), device=x.device, dtype=torch.bfloat16)
        ops.avgpool_fwd(_nhwc(x), y, N, H * W, C)
        ctx.shape = (N, C, H, W)
        return y

    @staticmethod
    def backward(ctx, dy):
        ops = _ext.ops()
        N, C, H, W = ctx.shape
        dx = torch.empty((N, C, H, W), device=dy.device, dtype=torch.bfloat16,
                         memory_format=torch.channels_last)
        ops.avgpool_bwd(dy.contiguous().to(torch.bfloat16), dx.permute(0, 2, 3, 1), N, H * W, C)
        return dx


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    if x.dtype != torch.bfloat16 or x.shape[1] % 8 != 0:
        return x.float().mean(dim=(2, 3)).to(x.dtype)
    return AvgPoolHipFn.apply(x)


class MaxPoolHipFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k: int, s: int, p: int):
        ops = _ext.ops()
        N, C, H, W = x.shape
        OH = (H + 2 * p - k) // s + 1
        OW = (W + 2 * p - k) // s + 1
        y = torch.empty((N, C, OH, OW), device=x.device, dtype=torch.bfloat16,
                        memory_format=torch.channels_last)
        arg = torch.empty((N, OH, OW, C), device=x.device, dtype=torch.uint8)
        ops.maxpool_fwd(_nhwc(x), y.permute(0, 2, 3, 1), arg, k, s, p)
        ctx.save_for_backward(arg)
        ctx.geom = (N, C, H, W, k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        ops = _ext.ops()
        (arg,) = ctx.saved_tensors
        N, C, H, W, k, s, p = ctx.geom
        dx = torch.empty((N, C, H, W), device=dy.device, dtype=torch.bfloat16,
                         memory_format=torch.channels_last)
        ops.maxpool_bwd(_nhwc(dy.to(torch.bfloat16)), arg, dx.permute(0, 2, 3, 1), k, s, p)
        return dx, None, None, None
