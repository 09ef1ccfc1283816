"""Autograd wrapper of the segmented SyncBN kernels (``csrc/bn.hip``).

Per layer and step: forward = [stats partials from the producing conv's epilogue, or a stats
pass] → reduce → (one all-reduce of [Σx; Σx²] for all views when distributed) → finalize
(mean/invstd, running stats, num_batches_tracked += views) → fused apply (affine + residual +
ReLU).  Backward = reduce (Σg, Σg·x̂ with the ReLU mask) → (one all-reduce) → finalize (dγ, dβ
written straight into the flat fp32 gradient buffer) → fused apply (dx, and d(residual) = g).
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist

from . import _ext
from ..parallel.state import site_key


def _rows(t: torch.Tensor) -> torch.Tensor:
    """[R, C] contiguous row view of a channels_last 4-D or a 2-D tensor."""
    if t.dim() == 4:
        if not t.is_contiguous(memory_format=torch.channels_last):
            t = t.contiguous(memory_format=torch.channels_last)
        return t.permute(0, 2, 3, 1).reshape(-1, t.shape[1])
    return t.contiguous()


def _empty_like_cl(x: torch.Tensor) -> torch.Tensor:
    if x.dim() == 4:
        return torch.empty(x.shape, device=x.device, dtype=x.dtype,
                           memory_format=torch.channels_last)
    return torch.empty_like(x)


def _allreduce(t: torch.Tensor, st) -> None:
    if st.comm:
        dist.all_reduce(t, group=st.stats_group)


def _grad_out(param: torch.Tensor):
    slot = getattr(param, "_slot", None)
    if slot is not None:
        return slot.grad, slot
    return torch.empty(param.shape, device=param.device, dtype=torch.float32), None


class BatchNormHipFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, residual, bn, segments, relu, st):
        ops = _ext.ops()
        S = segments
        C = x.shape[1]
        xr = _rows(x)
        R = xr.shape[0]
        dev = x.device
        pre = getattr(x, "_simclr_stats", None)
        if pre is not None and pre[1] % S == 0:
            partial, nblk_total = pre
            nblk = nblk_total // S
        else:
            nblk = ops.bn_blocks(R, C, S)
            partial = torch.empty((S * nblk * 2 * C,), device=dev, dtype=torch.float32)
            ops.bn_stats(xr, S, partial)
        count = float((R // S) * st.world_size)
        mi = torch.empty((2 * S * C,), device=dev, dtype=torch.float32)
        ipc = getattr(st, "ipc", None)
        if not st.comm or ipc is not None:  # one launch (the IPC exchange runs inside it)
            ops.bn_reduce_fused(partial, nblk, S, C, 1, None, count, bn.eps, bn.momentum,
                                bn.running_mean, bn.running_var, mi, bn.num_batches_tracked,
                                **(ipc.kwargs(site_key(bn, "fwd"), S, C) if ipc is not None else {}))
        else:
            stats = torch.empty((2 * S * C,), device=dev, dtype=torch.float32)
            ops.bn_reduce_fused(partial, nblk, S, C, 0, stats)
            _allreduce(stats, st)
            ops.bn_finalize(stats, S, C, count, bn.eps, bn.momentum, bn.running_mean,
                            bn.running_var, mi, bn.num_batches_tracked)
        y = _empty_like_cl(x)
        res_r = _rows(residual) if residual is not None else None
        ops.bn_apply(xr, res_r, _rows(y), mi, weight.detach(), bias.detach(), S, relu)
        ctx.save_for_backward(x, y if relu else None, mi, weight)
        ctx.cfg = (S, relu, residual is not None, count, st)
        ctx.bias = bias
        ctx.bn_key = site_key(bn, "bwd")  # the BatchNorm's IPC exchange site
        return y

    @staticmethod
    def backward(ctx, dy):
        ops = _ext.ops()
        x, y, mi, weight = ctx.saved_tensors
        S, relu, has_res, count, st = ctx.cfg
        C = x.shape[1]
        xr = _rows(x)
        R = xr.shape[0]
        dev = x.device
        dyr = _rows(dy)
        if dyr.dtype != torch.bfloat16:
            dyr = dyr.to(torch.bfloat16)
        yr = _rows(y) if y is not None else None
        nblk = ops.bn_blocks(R, C, S)
        partial = torch.empty((S * nblk * 2 * C,), device=dev, dtype=torch.float32)
        ops.bn_bwd_reduce(dyr, yr, xr, mi, S, relu, partial)
        dgamma, gslot = _grad_out(weight)
        dbeta, bslot = _grad_out(ctx.bias)
        coef = torch.empty((3 * S * C,), device=dev, dtype=torch.float32)
        ipc = getattr(st, "ipc", None)
        if not st.comm or ipc is not None:
            # with the IPC exchange the kernel writes dγ, dβ from the local sums and the
            # coefficients from the global ones
            ops.bn_reduce_fused(partial, nblk, S, C, 2, None, count, 0.0, 0.0, None, None, mi,
                                None, weight.detach(), None, None, dgamma, dbeta, coef,
                                **(ipc.kwargs(ctx.bn_key, S, C) if ipc is not None
                                   else {}))
        else:
            # dγ, dβ from the LOCAL sums (the data-parallel reducer sums them across ranks,
            # as SyncBatchNorm + DDP do); the input gradient needs the global sums
            sums = torch.empty((2 * S * C,), device=dev, dtype=torch.float32)
            ops.bn_reduce_fused(partial, nblk, S, C, 0, sums, dgamma=dgamma, dbeta=dbeta)
            _allreduce(sums, st)
            ops.bn_bwd_finalize(sums, mi, weight.detach(), S, C, count, None, None, coef)
        if gslot is not None:
            gslot.store.mark_ready(gslot.index)
        if bslot is not None:
            bslot.store.mark_ready(bslot.index)
        dx = _empty_like_cl(x)
        dres = _empty_like_cl(x) if has_res else None
        ops.bn_bwd_apply(dyr, yr, xr, coef, S, relu, _rows(dx),
                         _rows(dres) if dres is not None else None)
        gw = None if gslot is not None else dgamma
        gb = None if bslot is not None else dbeta
        return dx, gw, gb, dres, None, None, None, None


def batch_norm_train(x, bn, segments, residual, relu, st):
    if x.shape[1] % 8 != 0:
        raise ValueError(f"HIP BatchNorm needs channels % 8 == 0, got {x.shape[1]}")
    if residual is not None and residual.dtype != x.dtype:
        residual = residual.to(x.dtype)
    return BatchNormHipFn.apply(x, bn.weight, bn.bias, residual, bn, segments, relu, st)


def batch_norm_eval(x, bn, residual, relu):
    ops = _ext.ops()
    y = _empty_like_cl(x)
    ops.bn_apply_eval(_rows(x), _rows(residual) if residual is not None else None, _rows(y),
                      bn.running_mean, bn.running_var, bn.weight.detach(), bn.bias.detach(),
                      bn.eps, relu)
    return y
