"""Reference-semantics training step built only from stock torch ops (the throughput baseline).

This re-creates what the reference does per step (``/root/reference/main.py:104-122``):
torchvision-topology ResNet (model.py:76-114) with ``nn.BatchNorm2d`` (SyncBN when
distributed, main.py:176), two separate forwards (view0 then view1, main.py:112-113), the
NT-Xent of loss.py:33-65, SGD+LARC (Apex semantics, main.py:85-94; Apex is not installed so the
LARC step is written out with the same per-tensor Python loop) and the cosine/warmup LR.
It is used by ``bench.py --impl reference`` to measure the reference's images/sec on the same
hardware, since the reference publishes no throughput.
"""
from __future__ import annotations

import math
from collections import OrderedDict

import torch
from torch import nn
import torch.nn.functional as F


class _Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        idt = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        if self.downsample is not None:
            idt = self.downsample(x)
        return self.relu(out + idt)


class _Basic(nn.Module):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x):
        idt = x
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        if self.downsample is not None:
            idt = self.downsample(x)
        return self.relu(out + idt)


class PlainResNet(nn.Module):
    def __init__(self, base_cnn="resnet50", stem="imagenet", stem_padding=3):
        super().__init__()
        block, layers = ((_Bottleneck, [3, 4, 6, 3]) if base_cnn == "resnet50"
                         else (_Basic, [2, 2, 2, 2]))
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, 2, 3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make(block, 64, layers[0])
        self.layer2 = self._make(block, 128, layers[1], 2)
        self.layer3 = self._make(block, 256, layers[2], 2)
        self.layer4 = self._make(block, 512, layers[3], 2)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        if stem != "imagenet":
            self.conv1 = nn.Conv2d(3, 64, 3, 1, stem_padding if stem == "reference_cifar" else 1,
                                   bias=False)
            self.maxpool = nn.Identity()
        self.num_features = 512 * block.expansion

    def _make(self, block, planes, blocks, stride=1):
        ds = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            ds = nn.Sequential(nn.Conv2d(self.inplanes, planes * block.expansion, 1, stride,
                                         bias=False), nn.BatchNorm2d(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, ds)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)


class PlainContrastive(nn.Module):
    def __init__(self, base_cnn="resnet50", d=128, stem="imagenet"):
        super().__init__()
        self.f = PlainResNet(base_cnn, stem)
        H = self.f.num_features
        self.g = nn.Sequential(OrderedDict([
            ("linear1", nn.Linear(H, H)), ("bn1", nn.BatchNorm1d(H)), ("relu1", nn.ReLU()),
            ("linear2", nn.Linear(H, d, bias=False))]))

    def forward(self, x):
        return self.g(self.f(x))


def nt_xent_reference(view0, view1, temperature):
    """loss.py:33-65, reduction='mean'."""
    view0 = F.normalize(view0, p=2, dim=1)
    view1 = F.normalize(view1, p=2, dim=1)
    n = len(view0)
    targets = torch.arange(n, device=view0.device)
    mask = ~torch.eye(n, dtype=torch.bool, device=view0.device)
    sim00 = (view0 @ view0.t() / temperature)[mask].view(n, -1)
    sim11 = (view1 @ view1.t() / temperature)[mask].view(n, -1)
    sim01 = view0 @ view1.t() / temperature
    sim0 = torch.cat([sim01, sim00], dim=1)
    sim1 = torch.cat([sim01.t(), sim11], dim=1)
    loss = F.cross_entropy(sim0, targets, reduction="sum") + F.cross_entropy(sim1, targets,
                                                                           reduction="sum")
    return loss / n * 0.5


def exclude_from_wt_decay(named_params, weight_decay, skip_list=("bias", "bn")):
    params, excluded = [], []
    for name, p in named_params:
        if not p.requires_grad:
            continue
        (excluded if any(s in name for s in skip_list) else params).append(p)
    return [{"params": params, "weight_decay": weight_decay},
            {"params": excluded, "weight_decay": 0.0}]


@torch.no_grad()
def larc_step(optim: torch.optim.SGD, trust_coefficient=0.001, eps=1e-8):
    """Apex LARC(clip=False) semantics, written with the same per-tensor loop + host syncs."""
    wds = []
    for group in optim.param_groups:
        wd = group["weight_decay"]
        wds.append(wd)
        group["weight_decay"] = 0
        for p in group["params"]:
            if p.grad is None:
                continue
            param_norm = torch.norm(p.data)
            grad_norm = torch.norm(p.grad.data)
            if param_norm != 0 and grad_norm != 0:
                adaptive_lr = trust_coefficient * param_norm / (grad_norm + param_norm * wd + eps)
                p.grad.data += wd * p.data
                p.grad.data *= adaptive_lr
    optim.step()
    for group, wd in zip(optim.param_groups, wds):
        group["weight_decay"] = wd
