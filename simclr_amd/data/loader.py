"""Device-resident data pipeline: sharded sampler + on-GPU two-view augmentation.

Reference: ``DistributedSampler(shuffle=True)`` + ``DataLoader(batch_size=batches, num_workers=8,
pin_memory=True, drop_last=True)`` yielding ``((v0, v1), label)`` from PIL augmentation in CPU
worker processes (``/root/reference/main.py:156-173``).

Here the uint8 training set is uploaded to HBM once; per step the only host→device traffic is
the batch's index vector, and the ``augment`` HIP kernel writes both views straight into one
bf16 NHWC ``[2n, 8, H, W]`` tensor (view 0 rows first, channels zero-padded to 8 for the conv
gather) that the model consumes as a single ``segments=2`` forward.  The shard/shuffle order is
exactly ``torch.utils.data.DistributedSampler``'s (seed 0 + epoch, pad to a multiple of the
world size, rank-strided), with ``drop_last`` batching.  CPU tensors use the NumPy twin of the
kernel (``augment_ref``) and produce fp32 NCHW 3-channel views.
"""
from __future__ import annotations

from typing import Iterator, List, Optional, Tuple

import numpy as np
import torch

from . import augment_ref
from .datasets import ImageDataset

CPAD = 8


def shard_indices_tensor(n: int, epoch: int, rank: int, world: int, shuffle: bool = True,
                         seed: int = 0, drop_last: bool = False) -> torch.Tensor:
    """Identical index stream to ``DistributedSampler(...).set_epoch(epoch)`` iteration, as an
    int64 CPU tensor built with vectorised ops (no Python list of the permutation: ~0.3 ms for
    CIFAR's 50,000 indices, so an epoch rollover never stalls the host issue loop)."""
    if shuffle:
        g = torch.Generator()
        g.manual_seed(seed + epoch)
        indices = torch.randperm(n, generator=g)
    else:
        indices = torch.arange(n, dtype=torch.int64)
    if not drop_last:
        total = ((n + world - 1) // world) * world
        pad = total - n
        if pad:  # DistributedSampler repeats the head of the order (cyclically if pad > n)
            indices = torch.cat([indices, indices.repeat((pad + n - 1) // n)[:pad]])
    else:
        total = (n // world) * world
        indices = indices[:total]
    return indices[rank:total:world].contiguous()


def shard_indices(n: int, epoch: int, rank: int, world: int, shuffle: bool = True,
                  seed: int = 0, drop_last: bool = False) -> np.ndarray:
    """NumPy view of :func:`shard_indices_tensor` (reference ``DistributedSampler`` order)."""
    return shard_indices_tensor(n, epoch, rank, world, shuffle, seed, drop_last).numpy()


class ContrastiveLoader:
    """Iterates ``(x, labels)`` per step; x = both augmented views of the rank's batch."""

    def __init__(self, dataset: ImageDataset, batch_size: int, device: torch.device,
                 rank: int = 0, world: int = 1, strength: float = 0.5, seed: int = 0,
                 views: int = 2, out_size: Optional[int] = None, augment: bool = True,
                 shuffle: bool = True, drop_last: bool = True, sampler_seed: int = 0,
                 use_gpu_kernel: Optional[bool] = None):
        self.ds = dataset
        self.n = batch_size
        self.device = torch.device(device)
        self.rank, self.world = rank, world
        self.strength = strength
        self.seed = seed
        self.views = views
        self.H, self.W = dataset.images.shape[1], dataset.images.shape[2]
        self.OH = out_size or self.H
        self.OW = out_size or self.W
        self.augment = augment
        self.shuffle = shuffle
        self.drop_last = drop_last
        self.sampler_seed = sampler_seed
        self.epoch = 0
        self.counter = 0  # global step counter feeding the augmentation RNG
        if use_gpu_kernel is None:
            use_gpu_kernel = self.device.type == "cuda"
        self.gpu = use_gpu_kernel
        if self.gpu:
            from ..ops import _ext
            _ext.require()
            self.images = torch.from_numpy(dataset.images).to(self.device)
        else:
            self.images = dataset.images
        self.labels = torch.from_numpy(dataset.labels).to(self.device)
        # pre-training ignores the labels (no per-step label gather) and may hand the loader the
        # captured step's static input, so the augmentation writes straight into it (no copy)
        self.with_labels = True
        self.out: Optional[torch.Tensor] = None

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch

    def steps_per_epoch(self) -> int:
        per_rank = (len(self.ds) + self.world - 1) // self.world
        return per_rank // self.n if self.drop_last else (per_rank + self.n - 1) // self.n

    def __len__(self) -> int:
        return self.steps_per_epoch()

    def batch_from_indices(self, idx: torch.Tensor, counter: int) -> torch.Tensor:
        n = idx.numel()
        if self.gpu:
            shape = (self.views * n, CPAD, self.OH, self.OW)
            out = self.out
            if out is None or tuple(out.shape) != shape or not out.is_contiguous(
                    memory_format=torch.channels_last):
                out = torch.empty(shape, device=self.device, dtype=torch.bfloat16,
                                  memory_format=torch.channels_last)
            torch.ops.simclr_amd.augment(self.images, idx, n, self.views, self.OH, self.OW, CPAD,
                                         self.strength, self.seed, counter, 0,
                                         1 if self.augment else 0, out.permute(0, 2, 3, 1), None)
            return out
        arr = augment_ref.augment_batch(self.images, idx.cpu().numpy(), self.views, self.OH,
                                        self.OW, self.strength, self.seed, counter,
                                        augment=self.augment)
        return torch.from_numpy(arr)

    def epoch_indices(self) -> torch.Tensor:
        """This epoch's shard order on the loader's device.  On a GPU the order goes through a
        pinned staging buffer with a ``non_blocking`` copy: the upload is queued on the stream
        behind the previous epoch's last steps and the host never waits for the device (a
        pageable copy would drain the launch queue at every epoch rollover).  The pinned buffer
        comes from torch's caching host allocator, which keeps it alive until the copy's stream
        has passed it."""
        order = shard_indices_tensor(len(self.ds), self.epoch, self.rank, self.world,
                                     self.shuffle, self.sampler_seed)
        if self.device.type != "cuda":
            return order.to(self.device)
        staged = torch.empty(order.shape, dtype=order.dtype, pin_memory=True)
        staged.copy_(order)
        return staged.to(self.device, non_blocking=True)

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        idx_all = self.epoch_indices()
        steps = self.steps_per_epoch()
        for s in range(steps):
            idx = idx_all[s * self.n:(s + 1) * self.n]
            x = self.batch_from_indices(idx, self.counter)
            self.counter += 1
            yield x, (self.labels[idx] if self.with_labels else None)


class EvalLoader:
    """Un-augmented (ToTensor-only) batches in order, for feature extraction."""

    def __init__(self, dataset: ImageDataset, batch_size: int, device: torch.device,
                 use_gpu_kernel: Optional[bool] = None):
        self.inner = ContrastiveLoader(dataset, batch_size, device, views=1, augment=False,
                                       shuffle=False, drop_last=False,
                                       use_gpu_kernel=use_gpu_kernel)

    def __len__(self):
        return self.inner.steps_per_epoch()

    def __iter__(self):
        return iter(self.inner)
