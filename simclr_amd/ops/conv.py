"""Convolution front-end.

Reference: every conv in the reference is an implicit torchvision ``nn.Conv2d`` call
(``/root/reference/model.py:76-114``) dispatched to cuDNN in fp32 NCHW.

Here a ``Conv2d`` keeps fp32 master weights (views into the flat parameter store, see
``simclr_amd/parallel/flat.py``).  On the GPU fast path (bf16 NHWC activations) it runs the
hand-written implicit-GEMM kernels of ``csrc/conv.hip`` on the bf16 *shadow* copy of the weight
that the fused LARS kernel rewrites after every update (no per-step cast pass), and the weight
gradient is written as fp32 directly into the flat gradient buffer, which notifies the
data-parallel reducer.  fp32 / CPU tensors take ``torch.nn.functional.conv2d`` (the parity path).
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import nn
import torch.nn.functional as F


class ShadowWeight(torch.autograd.Function):
    """torch-path twin of the HIP plumbing: hand the compute op the low-precision shadow and
    route its gradient (upcast to fp32) into the flat gradient slot of the master parameter."""

    @staticmethod
    def forward(ctx, master: torch.Tensor, shadow: torch.Tensor, slot):  # noqa: D401
        ctx.slot = slot
        return shadow.view_as(shadow)

    @staticmethod
    def backward(ctx, grad):
        ctx.slot(grad)
        return None, None, None


class ParamSlot:
    """Per-parameter binding into the flat store: shadow view, grad view, reducer index.

    ``shadow``/``grad`` are in *storage* layout (OHWI for conv weights)."""

    __slots__ = ("shadow", "grad", "index", "store")

    def __init__(self, shadow: Optional[torch.Tensor], grad: torch.Tensor, index: int, store):
        self.shadow = shadow
        self.grad = grad
        self.index = index
        self.store = store

    def __call__(self, g: torch.Tensor) -> None:
        if g.dim() == 4 and self.grad.dim() == 4:
            g = g.permute(0, 2, 3, 1)  # OIHW grad -> OHWI storage
        self.grad.copy_(g.reshape(self.grad.shape) if g.shape != self.grad.shape else g)
        self.store.mark_ready(self.index)


def effective_weight(module: nn.Module, name: str = "weight") -> torch.Tensor:
    """The weight a torch compute op should consume (bf16 shadow when bound, else master)."""
    w = getattr(module, name)
    slot: Optional[ParamSlot] = getattr(w, "_slot", None)
    if slot is not None and slot.shadow is not None:
        sh = slot.shadow
        if sh.dim() == 4:
            sh = sh.permute(0, 3, 1, 2)  # OHWI storage -> OIHW logical
        if torch.is_grad_enabled() and w.requires_grad:
            return ShadowWeight.apply(w, sh, slot)
        return sh
    return w


class Conv2d(nn.Conv2d):
    """``nn.Conv2d`` with identical parameters/state-dict, MI355X compute path.

    ``emit_bn_stats``: the forward kernel also produces the BatchNorm statistics partials of its
    output (every conv of a ResNet feeds a BatchNorm)."""

    emit_bn_stats = True

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from . import registry
        if x.dtype == torch.bfloat16 and registry.use_hip(x):
            from . import conv_hip
            out = conv_hip.conv2d(x, None, self.stride, self.padding, weight_param=self.weight,
                                  emit_stats=self.emit_bn_stats and self.training)
            if out is not None:
                return out
        w = effective_weight(self)
        if w.dtype != x.dtype:
            w = w.to(x.dtype)
        ci = w.shape[1]
        if x.shape[1] != ci:  # channel-padded stem input (GPU augmentation writes 8 channels)
            x = x[:, :ci]
        return F.conv2d(x, w, None, self.stride, self.padding)
