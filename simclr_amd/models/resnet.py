"""ResNet-18/50 backbones with torchvision-compatible parameter names.

Parity target: the reference builds its backbone from ``torchvision.models.resnet18/50``
and then performs surgery on it (``/root/reference/model.py:76-114``):

* resnet18 + ``is_cifar``: ``conv1`` becomes ``Conv2d(3, 64, k=3, s=1, padding=3, bias=False)``
  (PyTorch default init, *not* torchvision's kaiming-normal) and ``maxpool`` becomes identity
  (model.py:99-104).
* resnet50 keeps the ImageNet 7x7/s2 stem + maxpool even on 32x32 inputs (model.py:90-92).
* ``fc`` becomes identity (model.py:111) for the contrastive model, or ``Linear(H, classes)``
  for the supervised model (model.py:164).

torchvision is not available in this environment, so the network is written here from scratch.
The module tree and parameter names are kept identical to torchvision's (``conv1``, ``bn1``,
``layer{1..4}.{i}.conv{1,2,3}``, ``...downsample.{0,1}``, ``fc``) so the reference checkpoint
format round-trips.  The initialisation matches torchvision's ``ResNet.__init__``:
kaiming-normal(fan_out, relu) for convs, BN gamma=1 / beta=0.

MI355X-first differences from the reference:

* Blocks call their norm layers with fused epilogue flags (``relu=``, ``residual=``), so
  BN-apply + residual add + ReLU is a single HIP kernel (see ``simclr_amd/ops/batchnorm.py``).
* The forward takes ``segments``: the two SimCLR views are pushed through ONE forward as a
  ``2N`` batch while BatchNorm statistics stay per view (reference semantics: two separate
  forwards, main.py:112-113).
* Extra opt-in knobs: ``cifar_stem`` (3x3/s1/p1 stem, no maxpool — the "CIFAR-ResNet-50" of the
  north star) and ``stem_padding``.
"""
from __future__ import annotations

import math
import os
from typing import Callable, List, Optional, Type

import torch
from torch import nn

from ..ops.batchnorm import BatchNorm2d, BatchNorm1d
from ..ops.conv import Conv2d
from ..ops.pooling import MaxPool2d
from .heads import Linear


def _kaiming_normal_fan_out_(w: torch.Tensor) -> None:
    nn.init.kaiming_normal_(w, mode="fan_out", nonlinearity="relu")


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes: int, planes: int, stride: int = 1,
                 downsample: Optional[nn.Module] = None):
        super().__init__()
        self.conv1 = Conv2d(inplanes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn1 = BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)  # kept for module-tree parity; fused into bn
        self.conv2 = Conv2d(planes, planes, 3, stride=1, padding=1, bias=False)
        self.bn2 = BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x: torch.Tensor, segments: int = 1) -> torch.Tensor:
        identity = x
        out = self.bn1(self.conv1(x), relu=True, segments=segments)
        out = self.conv2(out)
        if self.downsample is not None:
            identity = self.downsample[1](self.downsample[0](x), segments=segments)
        return self.bn2(out, residual=identity, relu=True, segments=segments)


class Bottleneck(nn.Module):
    """torchvision ResNet v1.5 bottleneck (stride on the 3x3 conv)."""
    expansion = 4

    def __init__(self, inplanes: int, planes: int, stride: int = 1,
                 downsample: Optional[nn.Module] = None):
        super().__init__()
        width = planes
        self.conv1 = Conv2d(inplanes, width, 1, bias=False)
        self.bn1 = BatchNorm2d(width)
        self.conv2 = Conv2d(width, width, 3, stride=stride, padding=1, bias=False)
        self.bn2 = BatchNorm2d(width)
        self.conv3 = Conv2d(width, planes * self.expansion, 1, bias=False)
        self.bn3 = BatchNorm2d(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x: torch.Tensor, segments: int = 1) -> torch.Tensor:
        identity = x
        out = self.bn1(self.conv1(x), relu=True, segments=segments)
        out = self.bn2(self.conv2(out), relu=True, segments=segments)
        out = self.conv3(out)
        if self.downsample is not None:
            identity = self.downsample[1](self.downsample[0](x), segments=segments)
        return self.bn3(out, residual=identity, relu=True, segments=segments)


class _Identity(nn.Module):
    def forward(self, x, *args, **kwargs):
        return x


class ResNet(nn.Module):
    def __init__(self, block: Type[nn.Module], layers: List[int], num_classes: Optional[int] = 1000,
                 stem: str = "imagenet", stem_padding: int = 3):
        """
        :param stem: ``imagenet`` (7x7/s2/p3 + maxpool, torchvision default),
                     ``reference_cifar`` (3x3/s1/p=stem_padding, no maxpool, default-init conv —
                     the reference's resnet18 surgery, model.py:99-104) or
                     ``cifar`` (3x3/s1/p1, no maxpool; opt-in CIFAR-ResNet).
        :param num_classes: ``None`` replaces ``fc`` with identity (model.py:111).
        """
        super().__init__()
        self.inplanes = 64
        self.stem = stem
        self.conv1 = Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool: nn.Module = MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.num_features = 512 * block.expansion
        self.fc: nn.Module = (Linear(self.num_features, num_classes)
                              if num_classes is not None else _Identity())

        # torchvision ResNet.__init__ initialisation
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                _kaiming_normal_fan_out_(m.weight)
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

        # stem surgery AFTER init, like the reference (replaced conv keeps PyTorch default init, Q8)
        if stem in ("reference_cifar", "cifar"):
            pad = stem_padding if stem == "reference_cifar" else 1
            self.conv1 = Conv2d(3, 64, kernel_size=3, stride=1, padding=pad, bias=False)
            self.maxpool = _Identity()
        elif stem != "imagenet":
            raise ValueError(f"unknown stem {stem!r}")

    def _make_layer(self, block, planes: int, blocks: int, stride: int = 1) -> nn.Sequential:
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                Conv2d(self.inplanes, planes * block.expansion, 1, stride=stride, bias=False),
                BatchNorm2d(planes * block.expansion),
            )
        layers = [block(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes))
        return nn.Sequential(*layers)

    # the fused stage executor (models/fused.py) runs layer1..layer4 in training on the HIP
    # path; ``use_fused_stages = False`` (or SIMCLR_FUSED=0) keeps the per-module path
    use_fused_stages = os.environ.get("SIMCLR_FUSED", "1") != "0"

    def _fused_executor(self, x: torch.Tensor, segments: int, check: bool = True):
        if not (self.training and self.use_fused_stages and torch.is_grad_enabled()
                and x.is_cuda and x.dtype == torch.bfloat16):
            return None
        from ..ops import registry
        if not registry.use_hip(x):
            return None
        from .fused import FusedStages
        cache = self.__dict__.setdefault("_fused_cache", {})
        ex = cache.get(segments)
        if ex is None:
            ex = cache[segments] = FusedStages(self, segments)
        return ex if (not check or ex.supported(x)) else None

    def forward_features(self, x: torch.Tensor, segments: int = 1) -> torch.Tensor:
        ex = self._fused_executor(x, segments, check=False)
        if ex is not None and ex.stem_supported(x):
            # stem + layer1..layer4 in the executor (models/fused.py stem_forward)
            from .fused import FusedStemStagesFn
            return global_avg_pool(FusedStemStagesFn.apply(x, self.conv1.weight, ex))
        x = self.bn1(self.conv1(x), relu=True, segments=segments)
        x = self.maxpool(x)
        ex = self._fused_executor(x, segments)
        if ex is not None:
            from .fused import FusedStagesFn
            x = FusedStagesFn.apply(x, self.layer1[0].conv1.weight, ex)
        else:
            for layer in (self.layer1, self.layer2, self.layer3, self.layer4):
                for blk in layer:
                    x = blk(x, segments=segments)
        return global_avg_pool(x)

    def forward(self, x: torch.Tensor, segments: int = 1) -> torch.Tensor:
        return self.fc(self.forward_features(x, segments=segments))


def global_avg_pool(x: torch.Tensor) -> torch.Tensor:
    """AdaptiveAvgPool2d(1) + flatten; fp32 accumulation of (possibly bf16) activations."""
    from ..ops import pooling
    return pooling.global_avg_pool(x)


def resnet18(num_classes: Optional[int] = 1000, **kw) -> ResNet:
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes=num_classes, **kw)


def resnet50(num_classes: Optional[int] = 1000, **kw) -> ResNet:
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes=num_classes, **kw)


def build_backbone(base_cnn: str, num_classes: Optional[int], is_cifar: bool = True,
                   cifar_stem: Optional[bool] = None, stem_padding: int = 3) -> ResNet:
    """Backbone exactly as the reference builds it (model.py:76-114), plus opt-in knobs.

    ``cifar_stem=None`` means reference behaviour: resnet18 gets the padding-3 CIFAR stem,
    resnet50 keeps the ImageNet stem.  ``cifar_stem=True`` gives a 3x3/s1/p1 stem
    to either network; ``False`` forces the ImageNet stem.
    """
    if base_cnn == "resnet18":
        ctor = resnet18
        default_stem = "reference_cifar" if is_cifar else "imagenet"
    elif base_cnn == "resnet50":
        ctor = resnet50
        default_stem = "imagenet"
    else:
        raise ValueError(
            "`base_cnn` must be either `resnet18` or `resnet50`. `{}` is unsupported.".format(base_cnn))
    if cifar_stem is None:
        stem = default_stem
    else:
        stem = "cifar" if cifar_stem else "imagenet"
    return ctor(num_classes=num_classes, stem=stem, stem_padding=stem_padding)
