"""Dense layers of the projection head on the MFMA implicit-GEMM kernels (a Linear is a 1x1
conv over an [M, 1, 1, K] "image"): forward with fused bias + BatchNorm-statistics epilogue,
dgrad against the transposed weight, split-M wgrad straight into the flat fp32 gradient, bias
gradient as a column sum.  (Reference: projection head ``/root/reference/model.py:65-70``,
SURVEY K6.)"""
from __future__ import annotations

from typing import Optional

import torch

from . import _ext
from .conv_hip import run_igemm, run_wgrad


def _geom(M, K, N):
    return [M, 1, 1, K, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, N, 1, 1, 1, 1, 0, 0, N]


def _weight_bf16(weight: torch.Tensor) -> torch.Tensor:
    slot = getattr(weight, "_slot", None)
    if slot is not None and slot.shadow is not None:
        return slot.shadow
    return weight.detach().to(torch.bfloat16).contiguous()


class LinearHipFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, emit_stats):
        ops = _ext.ops()
        M, K = x.shape
        N = weight.shape[0]
        xc = x.contiguous()
        w = _weight_bf16(weight)
        y = torch.empty((M, N), device=x.device, dtype=torch.bfloat16)
        b = bias.detach().float().contiguous() if bias is not None else None
        res = run_igemm(ops, xc, w, y, _geom(M, K, N), bias=b, want_stats=emit_stats)
        if res is not None:
            y._simclr_stats = res
        ctx.save_for_backward(xc, weight, bias)
        return y

    @staticmethod
    def backward(ctx, dy):
        ops = _ext.ops()
        x, weight, bias = ctx.saved_tensors
        M, K = x.shape
        N = weight.shape[0]
        dyc = dy.contiguous()
        if dyc.dtype != torch.bfloat16:
            dyc = dyc.to(torch.bfloat16)
        dx = None
        if ctx.needs_input_grad[0]:
            wt = torch.empty((K, N), device=dy.device, dtype=torch.bfloat16)
            ops.weight_transform(_weight_bf16(weight), wt, [N, 1, 1, K, 1, 1, 0, 1, 0, 1])
            dx = torch.empty((M, K), device=dy.device, dtype=torch.bfloat16)
            run_igemm(ops, dyc, wt, dx, _geom(M, N, K))
        dw = db = None
        if ctx.needs_input_grad[1]:
            g = _geom(M, K, N)
            slot = getattr(weight, "_slot", None)
            out = slot.grad if slot is not None else torch.empty(
                (N, K), device=dy.device, dtype=torch.float32)
            run_wgrad(ops, dyc, x, out, g, K)
            if slot is not None:
                slot.store.mark_ready(slot.index)
            else:
                dw = out
        if bias is not None and ctx.needs_input_grad[2]:
            bslot = getattr(bias, "_slot", None)
            out = bslot.grad if bslot is not None else torch.empty(
                (N,), device=dy.device, dtype=torch.float32)
            ops.colsum(dyc, out, 0.0)
            if bslot is not None:
                bslot.store.mark_ready(bslot.index)
            else:
                db = out
        return dx, dw, db, None


def linear(x: torch.Tensor, w: torch.Tensor, b: Optional[torch.Tensor],
           weight_param: Optional[torch.Tensor] = None, bias_param: Optional[torch.Tensor] = None,
           emit_stats: bool = True) -> Optional[torch.Tensor]:
    if x.dtype != torch.bfloat16 or x.dim() != 2:
        return None
    wp = weight_param if weight_param is not None else w
    N, K = wp.shape
    if N % 8 != 0 or K % 8 != 0:
        return None
    return LinearHipFn.apply(x, wp, bias_param if bias_param is not None else b, emit_stats)
