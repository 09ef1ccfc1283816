"""Cross-entropy + top-k accuracy and centroid class means on the HIP kernels of csrc/eval.hip
(SURVEY K10 / K11), with torch fallbacks off-GPU.

Reference: the probes compute ``F.cross_entropy`` and ``torch.topk`` per batch and pull every
count to the host (/root/reference/eval.py:78,104-136); ``CentroidClassifier.create_weights``
takes one masked mean per class (model.py:44-52).  Here one kernel gives per-row loss and the
target's rank (top-k correct ⇔ rank < k: no sort), counts stay on the device until the epoch
ends, and the class sums are one deterministic pass over the features.
"""
from __future__ import annotations

from typing import Tuple

import torch
import torch.nn.functional as F

from . import registry


def _hip_ok(logits: torch.Tensor) -> bool:
    return logits.is_cuda and registry.use_hip(logits) and logits.dim() == 2


def ce_rank(logits: torch.Tensor, y: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(per-row CE loss fp32, per-row rank of the target) — rank 0 means top-1 correct.

    Ties go to the lower class index; a NaN logit of another class ranks above the target (the
    order ``torch.topk`` uses) and a NaN target logit gets rank C, i.e. it is never correct."""
    logits = logits.float().contiguous()
    y = y.to(device=logits.device, dtype=torch.long).contiguous()
    if _hip_ok(logits):
        from . import _ext
        loss = torch.empty(logits.shape[0], device=logits.device, dtype=torch.float32)
        rank = torch.empty(logits.shape[0], device=logits.device, dtype=torch.int32)
        _ext.ops().ce_topk(logits, y, 0.0, loss, rank, None)
        return loss, rank
    loss = F.cross_entropy(logits, y, reduction="none")
    zt = logits.gather(1, y.view(-1, 1))
    idx = torch.arange(logits.shape[1], device=logits.device).view(1, -1)
    above = (logits > zt) | ((logits == zt) & (idx < y.view(-1, 1))) | \
        (torch.isnan(logits) & (idx != y.view(-1, 1)))  # torch.topk: NaN ranks above numbers
    rank = above.sum(1).to(torch.int32)
    # a NaN target logit (diverged probe, empty-class centroid) is never counted as correct
    return loss, torch.where(torch.isnan(zt.view(-1)), logits.shape[1], rank).to(torch.int32)


class _CEHipFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, y):
        from . import _ext
        B = logits.shape[0]
        loss = torch.empty(B, device=logits.device, dtype=torch.float32)
        rank = torch.empty(B, device=logits.device, dtype=torch.int32)
        dl = torch.empty_like(logits)
        _ext.ops().ce_topk(logits, y, 1.0 / B, loss, rank, dl)
        ctx.save_for_backward(dl)
        return loss.mean()

    @staticmethod
    def backward(ctx, g):
        (dl,) = ctx.saved_tensors
        return dl * g, None


def cross_entropy(logits: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """Mean cross-entropy (``F.cross_entropy`` semantics); on the GPU the forward kernel also
    produces the gradient, so the backward is a scale."""
    logits = logits.float().contiguous()
    y = y.to(device=logits.device, dtype=torch.long).contiguous()
    if _hip_ok(logits) and logits.requires_grad:
        return _CEHipFn.apply(logits, y)
    return F.cross_entropy(logits, y)


def class_means(X: torch.Tensor, y: torch.Tensor, num_classes: int) -> torch.Tensor:
    """[num_classes][D] per-class mean features (NaN rows for empty classes, as the reference's
    mean of an empty selection)."""
    y = y.to(device=X.device, dtype=torch.long).contiguous()
    if X.is_cuda and registry.use_hip(X) and num_classes <= 250:
        from . import _ext
        Xf = X.float().contiguous()
        sums = torch.empty(num_classes, X.shape[1], device=X.device, dtype=torch.float32)
        counts = torch.empty(num_classes, device=X.device, dtype=torch.float32)
        _ext.ops().class_sums(Xf, y, num_classes, sums, counts)
    else:
        sums = torch.zeros(num_classes, X.shape[1], dtype=torch.float64, device=X.device)
        sums.index_add_(0, y, X.double())
        counts = torch.bincount(y, minlength=num_classes).to(sums.dtype)
    means = (sums / counts.clamp_min(1)[:, None]).to(X.dtype)
    empty = counts == 0
    if bool(empty.any()):
        means[empty] = float("nan")
    return means
