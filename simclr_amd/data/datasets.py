"""Datasets: CIFAR-10/100 readers (no torchvision) and a deterministic synthetic generator.

Reference: ``torchvision.datasets.CIFAR10/100(root="~/pytorch_datasets", download=True)``
(``/root/reference/main.py:156-167``, eval.py:213-244).  There is no network here, so the reader
only loads data that is already on disk, from either the "python" pickled batches
(``cifar-10-batches-py`` / ``cifar-100-python``) or the binary release
(``cifar-10-batches-bin``); with ``synthetic=True`` (or when nothing is on disk and the caller
allows it) a synthetic dataset of the same shape is generated.

All datasets are returned as uint8 NHWC images + int64 labels so the whole training split can be
uploaded to HBM once (CIFAR-10: 150 MB) and augmented on device.
"""
from __future__ import annotations

import os
import pickle
from dataclasses import dataclass
from pathlib import Path
from typing import Optional

import numpy as np
import torch

DEFAULT_ROOT = "~/pytorch_datasets"


@dataclass
class ImageDataset:
    images: np.ndarray   # uint8 [N, H, W, 3]
    labels: np.ndarray   # int64 [N]
    num_classes: int
    name: str
    synthetic: bool = False

    def __len__(self) -> int:
        return len(self.labels)

    @property
    def data(self):  # torchvision attribute name used by the reference (main.py:74)
        return self.images


def _load_pickle(path: Path) -> dict:
    with open(path, "rb") as f:
        return pickle.load(f, encoding="bytes")  # user-provided dataset file (CIFAR format)


def _cifar_py(root: Path, name: str, train: bool) -> Optional[ImageDataset]:
    if name == "cifar10":
        d = root / "cifar-10-batches-py"
        files = [d / f"data_batch_{i}" for i in range(1, 6)] if train else [d / "test_batch"]
        key, ncls = b"labels", 10
    else:
        d = root / "cifar-100-python"
        files = [d / ("train" if train else "test")]
        key, ncls = b"fine_labels", 100
    if not all(f.exists() for f in files):
        return None
    xs, ys = [], []
    for f in files:
        e = _load_pickle(f)
        xs.append(np.asarray(e[b"data"], dtype=np.uint8).reshape(-1, 3, 32, 32))
        ys.append(np.asarray(e[key], dtype=np.int64))
    x = np.concatenate(xs).transpose(0, 2, 3, 1).copy()
    return ImageDataset(x, np.concatenate(ys), ncls, name)


def _cifar_bin(root: Path, name: str, train: bool) -> Optional[ImageDataset]:
    if name != "cifar10":
        d = root / "cifar-100-binary"
        files = [d / ("train.bin" if train else "test.bin")]
        rec, lab_off, ncls = 3074, 1, 100
    else:
        d = root / "cifar-10-batches-bin"
        files = ([d / f"data_batch_{i}.bin" for i in range(1, 6)] if train
                 else [d / "test_batch.bin"])
        rec, lab_off, ncls = 3073, 0, 10
    if not all(f.exists() for f in files):
        return None
    raw = np.concatenate([np.fromfile(f, dtype=np.uint8) for f in files]).reshape(-1, rec)
    labels = raw[:, lab_off].astype(np.int64)
    x = raw[:, rec - 3072:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1).copy()
    return ImageDataset(x, labels, ncls, name)


def synthetic_dataset(n: int, num_classes: int = 10, size: int = 32, seed: int = 0,
                      name: str = "synthetic", template_seed: int = 1234, noise: float = 25.0,
                      colour: bool = True) -> ImageDataset:
    """Class-structured random images: per-class colour/frequency template + per-image noise,
    so that learned features are non-trivially separable (used when no data is on disk).
    ``colour=False`` gives every class the same mean colour (texture is the only cue) and a
    larger ``noise`` makes the task harder (tools/e2e_probe.sh)."""
    g = np.random.default_rng(seed)
    labels = g.integers(0, num_classes, size=n).astype(np.int64)
    yy, xx = np.meshgrid(np.linspace(0, 1, size), np.linspace(0, 1, size), indexing="ij")
    tmpl = np.empty((num_classes, size, size, 3), dtype=np.float32)
    cg = np.random.default_rng(template_seed)  # shared by train and test splits
    for c in range(num_classes):
        col = cg.uniform(40, 215, size=3)
        if not colour:
            col = np.full(3, 128.0)
        fy, fx = cg.uniform(1, 4, size=2)
        ph = cg.uniform(0, 2 * np.pi)
        pat = np.sin(2 * np.pi * (fy * yy + fx * xx) + ph)
        tmpl[c] = col[None, None, :] + 35.0 * pat[..., None]
    imgs = np.empty((n, size, size, 3), dtype=np.uint8)
    bs = 4096
    for s in range(0, n, bs):
        e = min(n, s + bs)
        eps = g.normal(0, noise, size=(e - s, size, size, 3)).astype(np.float32)
        imgs[s:e] = np.clip(tmpl[labels[s:e]] + eps, 0, 255).astype(np.uint8)
    return ImageDataset(imgs, labels, num_classes, name, synthetic=True)


def synthetic_texture_dataset(n: int, num_classes: int = 10, size: int = 32, seed: int = 0,
                              name: str = "synthetic-texture", template_seed: int = 4321,
                              noise: float = 40.0) -> ImageDataset:
    """A mid-difficulty accuracy proxy (no CIFAR on the machine): the class is a texture — a
    sum of two oriented sinusoidal gratings with class-specific frequencies / orientations —
    while everything SimCLR's augmentations randomise is nuisance: a random mean colour per
    image (colour jitter / grayscale), a random phase and position (crop), a random contrast,
    plus Gaussian pixel noise (``noise``).  Orientations are chosen flip-symmetric per class
    (each class holds a grating and its mirror image), so horizontal flips keep the class.
    A probe must read texture frequency / orientation through noise: random-init features
    separate it only partly, and pre-training has to learn the invariances
    (tools/accuracy_proxy.sh, profiles/r6_accuracy_proxy.md)."""
    g = np.random.default_rng(seed)
    labels = g.integers(0, num_classes, size=n).astype(np.int64)
    cg = np.random.default_rng(template_seed)  # shared by the train and test splits
    freq = cg.uniform(1.5, 5.0, size=(num_classes, 2))       # cycles per image
    theta = cg.uniform(0.0, np.pi / 2, size=(num_classes, 2))
    yy, xx = np.meshgrid(np.arange(size) / size, np.arange(size) / size, indexing="ij")
    imgs = np.empty((n, size, size, 3), dtype=np.uint8)
    bs = 2048
    for s in range(0, n, bs):
        e = min(n, s + bs)
        m = e - s
        lab = labels[s:e]
        acc = np.zeros((m, size, size), dtype=np.float32)
        for k in range(2):
            th = theta[lab, k] * np.where(g.random(m) < 0.5, 1.0, -1.0)  # mirror pairs
            f = freq[lab, k] * g.uniform(0.85, 1.15, size=m)
            ph = g.uniform(0, 2 * np.pi, size=m)
            u = (np.cos(th)[:, None, None] * xx[None] + np.sin(th)[:, None, None] * yy[None])
            acc += np.sin(2 * np.pi * f[:, None, None] * u + ph[:, None, None])
        amp = g.uniform(18.0, 45.0, size=(m, 1, 1, 1)).astype(np.float32)
        col = g.uniform(60.0, 195.0, size=(m, 1, 1, 3)).astype(np.float32)
        tint = g.uniform(0.6, 1.0, size=(m, 1, 1, 3)).astype(np.float32)
        eps = g.normal(0, noise, size=(m, size, size, 3)).astype(np.float32)
        img = col + amp * tint * acc[..., None] + eps
        imgs[s:e] = np.clip(img, 0, 255).astype(np.uint8)
    return ImageDataset(imgs, labels, num_classes, name, synthetic=True)


def load_dataset(name: str, train: bool = True, root: str = DEFAULT_ROOT,
                 synthetic: bool = False, synthetic_size: Optional[int] = None,
                 allow_synthetic_fallback: bool = False, seed: int = 0,
                 image_size: int = 32, synthetic_noise: float = 25.0,
                 synthetic_colour: bool = True, synthetic_kind: str = "template") -> ImageDataset:
    name = name.lower()
    if name not in ("cifar10", "cifar100"):
        raise ValueError("experiment.name must be cifar10 or cifar100, got {!r}".format(name))
    ncls = 10 if name == "cifar10" else 100
    if not synthetic:
        r = Path(os.path.expanduser(root))
        for reader in (_cifar_py, _cifar_bin):
            ds = reader(r, name, train)
            if ds is not None:
                return ds
        if not allow_synthetic_fallback:
            raise FileNotFoundError(
                f"{name} not found under {r} (no network to download it); "
                "place the CIFAR python/binary batches there or run with data.synthetic=true")
    n = synthetic_size if synthetic_size is not None else (50000 if train else 10000)
    if synthetic_kind == "texture":
        return synthetic_texture_dataset(n, ncls, size=image_size,
                                         seed=seed + (0 if train else 7919),
                                         name=f"synthetic-texture-{name}", noise=synthetic_noise)
    if synthetic_kind != "template":
        raise ValueError(f"data.synthetic_kind must be template or texture, not {synthetic_kind!r}")
    return synthetic_dataset(n, ncls, size=image_size, seed=seed + (0 if train else 7919),
                             name=f"synthetic-{name}", noise=synthetic_noise,
                             colour=synthetic_colour)
