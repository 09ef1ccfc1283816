"""Projection head and downstream classifiers.

Parity: ``ProjectionHead`` (``/root/reference/model.py:56-73``), ``LinearClassifier``
(model.py:7-21), ``CentroidClassifier`` (model.py:24-53).  ``NonLinearClassifier`` is imported
by the reference's eval.py (eval.py:16,304) but never defined; it is
implemented here as Linear(F,F) → BN1d → ReLU → Linear(F,C), mirroring the projection head
(an inferred design, documented as such).
"""
from __future__ import annotations

import os
from collections import OrderedDict

import torch
from torch import nn
import torch.nn.functional as F

from ..ops.batchnorm import BatchNorm1d
from ..ops.conv import effective_weight


class Linear(nn.Linear):
    """``nn.Linear`` with the bf16-shadow / flat-gradient plumbing of ``ops.conv``.

    ``emit_bn_stats``: the GEMM epilogue also emits the statistics partials for a following
    BatchNorm1d (true for ``linear1`` of the heads)."""

    emit_bn_stats = False

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from ..ops import linear as linear_ops
        return linear_ops.linear_module(self, x)


class _MLP(nn.Module):
    """Linear → BN1d → ReLU → Linear with the fused BN+ReLU epilogue."""

    def __init__(self, in_features: int, hidden: int, out_features: int, last_bias: bool,
                 attr: str):
        super().__init__()
        lin1 = Linear(in_features, hidden)
        lin1.emit_bn_stats = True
        seq = nn.Sequential(OrderedDict([
            ("linear1", lin1),
            ("bn1", BatchNorm1d(hidden)),
            ("relu1", nn.ReLU()),
            ("linear2", Linear(hidden, out_features, bias=last_bias)),
        ]))
        self._attr = attr
        setattr(self, attr, seq)

    @property
    def _seq(self) -> nn.Sequential:
        return getattr(self, self._attr)

    # the fused GEMM-BN-GEMM schedule (models/head_fused.py) for eligible training batches
    # (SIMCLR_FUSED_HEAD=0: the per-op head, for A/B attribution)
    use_fused = os.environ.get("SIMCLR_FUSED_HEAD", "1") != "0"

    def forward(self, x: torch.Tensor, segments: int = 1) -> torch.Tensor:
        s = self._seq
        if self.training and self.use_fused and x.is_cuda:
            from .head_fused import fused_mlp
            out = fused_mlp(self, x, segments)
            if out is not None:
                return out
        h = s.linear1(x)
        h = s.bn1(h, relu=True, segments=segments)
        return s.linear2(h)

    @property
    def in_features(self) -> int:
        return self._seq.linear1.in_features

    @property
    def out_features(self) -> int:
        return self._seq.linear2.out_features


class ProjectionHead(_MLP):
    """g(h) = W2 · ReLU(BN(W1 h + b1)); keys ``projection_head.{linear1,bn1,linear2}.*``."""

    def __init__(self, num_last_hidden_units: int, d: int):
        super().__init__(num_last_hidden_units, num_last_hidden_units, d, last_bias=False,
                         attr="projection_head")


class NonLinearClassifier(_MLP):
    def __init__(self, num_features: int = 128, num_classes: int = 10):
        super().__init__(num_features, num_features, num_classes, last_bias=True,
                         attr="classifier")


class LinearClassifier(nn.Module):
    def __init__(self, num_features: int = 128, num_classes: int = 10):
        super().__init__()
        self.classifier = nn.Linear(num_features, num_classes)

    def forward(self, inputs: torch.Tensor, segments: int = 1) -> torch.Tensor:
        return self.classifier(inputs)


class CentroidClassifier(nn.Module):
    """Dot-product against per-class mean features (unnormalised, model.py:24-53)."""

    def __init__(self, weights: torch.Tensor):
        super().__init__()
        self.weights = weights  # d x num_classes

    def forward(self, inputs: torch.Tensor, segments: int = 1) -> torch.Tensor:
        return torch.matmul(inputs.to(self.weights.dtype), self.weights)

    @staticmethod
    def create_weights(dataset, num_classes: int) -> torch.Tensor:
        """Per-class means as one segmented reduction (HIP class-sum kernel on the GPU, K11)
        instead of C masked means; classes with no samples give NaN, as the reference's mean of
        an empty selection."""
        from ..ops.classify import class_means
        return class_means(dataset.data, dataset.targets, num_classes).t().contiguous()
