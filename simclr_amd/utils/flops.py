"""Model FLOPs of one SimCLR training step (utilisation accounting for bench.py).

The forward FLOPs are counted, not estimated: a CPU fp32 copy of the same architecture runs
one image per view through ``torch.utils.flop_counter.FlopCounterMode`` (every aten convolution
and matmul at its real shape, 2·M·N·K), and the count is scaled to the batch.  A training step is
taken as 3x the forward — forward, input gradient and weight gradient, the usual MFU convention —
so the number is comparable across implementations (the stem's unneeded input gradient and the
elementwise / BatchNorm / loss work are not subtracted / added; they are < 1 % either way).

ResNet-50 with the CIFAR stem at 32x32: 2 x 1.30 GFLOP per image and view in the forward, so
1,024 view-rows x 2.6 GFLOP x 3 = 8.0 TFLOP per 512-image step.
"""
from __future__ import annotations

from functools import lru_cache

import torch


@lru_cache(maxsize=None)
def forward_flops_per_image(model: str, cifar_stem, size: int, d: int = 128) -> int:
    """Forward FLOPs of one image through backbone + projection head (one view)."""
    from torch.utils.flop_counter import FlopCounterMode
    from ..models.contrastive import ContrastiveModel
    m = ContrastiveModel(base_cnn=model, d=d, cifar_stem=cifar_stem).eval()
    x = torch.zeros(1, 3, size, size)
    with torch.no_grad(), FlopCounterMode(display=False) as fc:
        m(x)
    return int(fc.get_total_flops())


def step_flops(model: str, cifar_stem, size: int, batch: int, views: int = 2,
               d: int = 128) -> int:
    """Model FLOPs of one training step of ``batch`` images x ``views`` views on one GPU."""
    return 3 * views * batch * forward_flops_per_image(model, cifar_stem, size, d)
