"""SimCLR model wrappers.

Parity: ``ContrastiveModel`` (``/root/reference/model.py:76-129``) with ``f`` (backbone, fc =
identity) and ``g`` (projection head), ``encode`` → h, ``forward`` → z; ``SupervisedModel``
(model.py:132-168) with ``f.fc = Linear(H, num_classes)``.

Both accept ``segments`` so the two augmented views can share one forward while BatchNorm
statistics remain per view.
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import nn

from ..parallel.state import tag_sites
from .heads import ProjectionHead
from .resnet import build_backbone


class ContrastiveModel(nn.Module):
    def __init__(self, base_cnn: str = "resnet18", d: int = 128, is_cifar: bool = True,
                 cifar_stem: Optional[bool] = None, stem_padding: int = 3):
        super().__init__()
        assert base_cnn in {"resnet18", "resnet50"}
        self.f = build_backbone(base_cnn, num_classes=None, is_cifar=is_cifar,
                                cifar_stem=cifar_stem, stem_padding=stem_padding)
        num_last_hidden_units = self.f.num_features
        self.g = ProjectionHead(num_last_hidden_units, d)
        tag_sites(self)  # stable IPC exchange-site names (comm/ipc.py)

    def encode(self, inputs: torch.Tensor, segments: int = 1) -> torch.Tensor:
        return self.f(inputs, segments=segments)  # N x H

    def forward(self, inputs: torch.Tensor, segments: int = 1) -> torch.Tensor:
        h = self.encode(inputs, segments=segments)
        return self.g(h, segments=segments)  # N x d


class SupervisedModel(nn.Module):
    def __init__(self, base_cnn: str = "resnet18", num_classes: int = 10, is_cifar: bool = True,
                 cifar_stem: Optional[bool] = None, stem_padding: int = 3):
        super().__init__()
        assert base_cnn in {"resnet18", "resnet50"}
        self.f = build_backbone(base_cnn, num_classes=num_classes, is_cifar=is_cifar,
                                cifar_stem=cifar_stem, stem_padding=stem_padding)
        tag_sites(self)

    def forward(self, inputs: torch.Tensor, segments: int = 1) -> torch.Tensor:
        return self.f(inputs, segments=segments)
