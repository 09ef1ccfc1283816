"""Cross-replica, per-view ("segmented") BatchNorm with fused residual-add + ReLU epilogue.

Reference semantics (``/root/reference/main.py:112-113,176``):
the reference converts every BN to ``SyncBatchNorm`` and calls the model twice per step (view0,
then view1), so each BN layer normalises each view with statistics over that view's *global*
batch (all ranks), and updates running statistics twice per step (momentum 0.1, unbiased
running variance with the global count, ``num_batches_tracked += 2``).

MI355X design: both views go through one forward as a ``S*n`` batch (``segments=S``).  Per
layer the GPU path runs

    fwd:  bn_stats (per-view per-channel Σx, Σx² partials) → [one RCCL all-reduce of
          S·2·C floats for *both* views] → bn_finalize (mean/invstd + running stats) →
          bn_apply (normalise + affine + residual + ReLU, bf16 NHWC out)
    bwd:  bn_bwd_reduce (Σg, Σg·x̂ with the ReLU mask from y) → [one all-reduce] →
          bn_bwd_finalize (dγ, dβ straight into the flat fp32 grad buffer) → bn_bwd_apply

i.e. 2 collectives per layer per step instead of the reference's 4 (2 forwards × gather +
2 backward all-reduces) and no separate ReLU/add kernels.  The CPU / ``backend=torch`` path is
a readable composition of torch ops with identical math, used as the numerics oracle.
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import nn

from . import registry


def _acc(t: torch.Tensor) -> torch.Tensor:
    """Accumulation precision of the torch oracles: fp32, or fp64 when the input is fp64 (the
    multi-process equivalence tests run in fp64 so that summation-order noise cannot hide a
    semantic difference)."""
    return t if t.dtype == torch.float64 else t.float()


class _BatchNormBase(nn.Module):
    def __init__(self, num_features: int, eps: float = 1e-5, momentum: float = 0.1):
        super().__init__()
        self.num_features = num_features
        self.eps = eps
        self.momentum = momentum
        self.weight = nn.Parameter(torch.ones(num_features))
        self.bias = nn.Parameter(torch.zeros(num_features))
        self.register_buffer("running_mean", torch.zeros(num_features))
        self.register_buffer("running_var", torch.ones(num_features))
        self.register_buffer("num_batches_tracked", torch.tensor(0, dtype=torch.long))

    def extra_repr(self) -> str:
        return f"{self.num_features}, eps={self.eps}, momentum={self.momentum}"

    def forward(self, x: torch.Tensor, residual: Optional[torch.Tensor] = None,
                relu: bool = False, segments: int = 1) -> torch.Tensor:
        if self.training:
            return registry.batch_norm_train(
                x, self, segments=segments, residual=residual, relu=relu)
        return registry.batch_norm_eval(x, self, residual=residual, relu=relu)


class BatchNorm2d(_BatchNormBase):
    """Drop-in for ``nn.BatchNorm2d``/``SyncBatchNorm`` (same parameters and buffers)."""


class BatchNorm1d(_BatchNormBase):
    """Drop-in for ``nn.BatchNorm1d`` on [N, C] inputs (projection head, model.py:67)."""


def reference_batch_norm_train(x: torch.Tensor, bn: _BatchNormBase, segments: int,
                               residual: Optional[torch.Tensor], relu: bool,
                               group=None, world_size: int = 1) -> torch.Tensor:
    """Oracle: torch-op composition of segmented SyncBN + residual + ReLU (differentiable).

    Statistics are fp32 sums; the cross-rank combine is a differentiable all-reduce of
    [Σx, Σx²] for all views at once (equal per-rank counts make this identical to SyncBN's
    count-weighted gather/combine).
    """
    N, C = x.shape[0], x.shape[1]
    assert N % segments == 0, f"batch {N} not divisible into {segments} views"
    n = N // segments
    chan_last = x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last) \
        and not x.is_contiguous()
    xf = _acc(x).reshape(segments, n, C, -1)
    L = xf.shape[-1]
    s1 = xf.sum(dim=(1, 3))
    s2 = (xf * xf).sum(dim=(1, 3))
    stats = torch.stack([s1, s2])  # [2, S, C]
    count = n * L
    if world_size > 1:
        from torch.distributed.nn.functional import all_reduce
        stats = all_reduce(stats, group=group)
        count *= world_size
    mean = stats[0] / count
    var = (stats[1] / count - mean * mean).clamp_min(0.0)
    invstd = torch.rsqrt(var + bn.eps)
    w = _acc(bn.weight)
    b = _acc(bn.bias)
    y = (xf - mean[:, None, :, None]) * (invstd * w)[:, None, :, None] + b[None, None, :, None]
    y = y.reshape(x.shape)
    if residual is not None:
        y = y + _acc(residual)
    if relu:
        y = torch.relu(y)
    with torch.no_grad():
        m = bn.momentum
        unbias = count / max(count - 1, 1)
        for s in range(segments):  # sequential updates == the reference's two forwards
            bn.running_mean.mul_(1 - m).add_(mean[s].detach() * m)
            bn.running_var.mul_(1 - m).add_(var[s].detach() * unbias * m)
            bn.num_batches_tracked.add_(1)
    y = y.to(x.dtype)
    if chan_last:
        y = y.contiguous(memory_format=torch.channels_last)
    return y


def reference_batch_norm_eval(x: torch.Tensor, bn: _BatchNormBase,
                              residual: Optional[torch.Tensor], relu: bool) -> torch.Tensor:
    C = x.shape[1]
    shape = (1, C) + (1,) * (x.dim() - 2)
    invstd = torch.rsqrt(_acc(bn.running_var) + bn.eps)
    scale = (_acc(bn.weight) * invstd).reshape(shape)
    shift = (_acc(bn.bias) - _acc(bn.running_mean) * _acc(bn.weight) * invstd).reshape(shape)
    y = _acc(x) * scale + shift
    if residual is not None:
        y = y + _acc(residual)
    if relu:
        y = torch.relu(y)
    y = y.to(x.dtype)
    if x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last):
        y = y.contiguous(memory_format=torch.channels_last)
    return y
