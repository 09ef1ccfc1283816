"""Downstream probes on frozen features: centroid, linear and nonlinear classifiers.

Parity: ``centroid_eval`` (``/root/reference/eval.py:61-85``), ``learnable_eval``
(eval.py:88-190) and the results-dict schema of eval.py:279-319:

* centroid: class-mean weights (unnormalised) · dot-product scores, top-1 / top-k accuracy;
* linear / nonlinear: SGD(lr = lr·batches/256, momentum, **nesterov=True**, wd = decay),
  ``CosineAnnealingLR(T_max = epochs·ceil(N/batches))`` stepped every batch, shuffled batches;
  after every epoch train and val (top-1, top-k, mean CE) are recomputed; the JSON reports the
  per-epoch lists and ``lowest_val_loss``, ``highest_val_acc``, ``highest_val_top_k_acc``.

Fixed reference defects: ``top_k <= 1`` no longer accumulates cumulative top-1 counts (Q4), and
``NonLinearClassifier`` exists (Q1).  Features and labels stay on the device; batches are index
permutations (no per-batch host copies).
"""
from __future__ import annotations

import logging
import math
from dataclasses import dataclass
from typing import Dict, List, Tuple

import torch
import torch.nn.functional as F

from ..models.heads import CentroidClassifier, LinearClassifier, NonLinearClassifier
from ..ops.classify import ce_rank, cross_entropy
from ..optim.schedule import cosine_lr

log = logging.getLogger(__name__)


@dataclass
class DownstreamDataset:
    """(data, targets) tensor dataset over extracted features (reference dataset.py:5-16)."""
    data: torch.Tensor
    targets: torch.Tensor

    def __post_init__(self):
        assert len(self.data) == len(self.targets)

    def __len__(self) -> int:
        return len(self.data)

    def __getitem__(self, i):
        return self.data[i], self.targets[i]


def _batches(n: int, bs: int, shuffle: bool, gen: torch.Generator, device):
    if shuffle:
        perm = torch.randperm(n, generator=gen).to(device)
    else:
        perm = torch.arange(n, device=device)
    for s in range(0, n, bs):
        yield perm[s:s + bs]


def _topk_correct(scores: torch.Tensor, y: torch.Tensor, top_k: int) -> Tuple[int, int]:
    """(top-1, top-k) correct counts: the target's rank (classes scoring above it) < k."""
    _, rank = ce_rank(scores, y)
    k = max(1, min(top_k, scores.shape[1]))
    return int((rank == 0).sum().item()), int((rank < k).sum().item())


@torch.no_grad()
def centroid_eval(ds: DownstreamDataset, classifier: CentroidClassifier, top_k: int = 5,
                  batch_size: int = 4096) -> Tuple[float, float]:
    _, c1, ck = _eval_counts(classifier, ds, top_k, batch_size, with_loss=False)
    return c1, ck


def _eval_counts(classifier, ds: DownstreamDataset, top_k: int, batch_size: int,
                 with_loss: bool = True) -> Tuple[float, float, float]:
    """Mean CE, top-1 and top-k accuracy over ``ds``, accumulated on the device (one host sync
    per call instead of three per batch, reference eval.py:104-136)."""
    n = len(ds)
    k = None
    acc = None
    for s in range(0, n, batch_size):
        x = ds.data[s:s + batch_size]
        y = ds.targets[s:s + batch_size].to(x.device)
        out = classifier(x).float()
        if k is None:
            k = max(1, min(top_k, out.shape[1]))
            acc = torch.zeros(3, dtype=torch.float64, device=out.device)
        loss, rank = ce_rank(out, y)
        acc[0] += loss.double().sum() if with_loss else 0.0
        acc[1] += (rank == 0).sum()
        acc[2] += (rank < k).sum()
    a = acc.cpu().tolist() if acc is not None else [0.0, 0.0, 0.0]
    return a[0] / n, a[1] / n, a[2] / n


@torch.no_grad()
def accuracies_loss(classifier, ds: DownstreamDataset, top_k: int = 5,
                    batch_size: int = 4096) -> Tuple[float, float, float]:
    classifier.eval()
    loss, c1, ck = _eval_counts(classifier, ds, top_k, batch_size)
    return c1, ck, loss


def learnable_eval(cfg, classifier, train: DownstreamDataset, val: DownstreamDataset,
                   top_k: int = 5, seed: int = 0) -> Tuple[List[float], ...]:
    p, e = cfg["parameter"], cfg["experiment"]
    epochs = p["epochs"]
    bs = e["batches"]
    n = len(train)
    total_steps = epochs * int(math.ceil(n / bs))
    if p["linear_schedule"]:
        lr0 = e["lr"] * bs / 256.0
    else:
        lr0 = e["lr"] * math.sqrt(bs)
    opt = torch.optim.SGD(classifier.parameters(), lr=lr0, momentum=p["momentum"], nesterov=True,
                          weight_decay=e["decay"])
    gen = torch.Generator()
    gen.manual_seed(seed)
    step = 0
    tr_acc, tr_topk, tr_loss, va_acc, va_topk, va_loss = [], [], [], [], [], []
    dev = train.data.device
    for epoch in range(1, epochs + 1):
        classifier.train()
        sum_loss = 0.0
        for idx in _batches(n, bs, True, gen, dev):
            for g in opt.param_groups:
                g["lr"] = cosine_lr(step, lr0, total_steps)
            x = train.data[idx]
            y = train.targets[idx].to(dev)
            opt.zero_grad()
            out = classifier(x).float()
            loss = cross_entropy(out, y)
            loss.backward()
            opt.step()
            step += 1
            sum_loss = sum_loss + loss.detach() * len(y)  # device-side: no sync per batch
        logging.info("Epoch:{}/{} progress:{:.3f} loss:{:.3f}, lr:{:.7f}".format(
            epoch, epochs, epoch / epochs, float(sum_loss) / n, cosine_lr(step, lr0, total_steps)))
        a, b, c = accuracies_loss(classifier, train, top_k)
        tr_acc.append(a)
        tr_topk.append(b)
        tr_loss.append(c)
        a, b, c = accuracies_loss(classifier, val, top_k)
        va_acc.append(a)
        va_topk.append(b)
        va_loss.append(c)
    return tr_acc, tr_topk, tr_loss, va_acc, va_topk, va_loss


def run_probe(cfg, kind: str, train: DownstreamDataset, val: DownstreamDataset, num_classes: int,
              top_k: int, device) -> Dict:
    if kind == "centroid":
        clf = CentroidClassifier(CentroidClassifier.create_weights(train, num_classes).to(device))
        train_acc, train_topk = centroid_eval(train, clf, top_k)
        val_acc, val_topk = centroid_eval(val, clf, top_k)
        logging.info("train acc: {}, val acc: {}".format(train_acc, val_acc))
        return {
            "train_acc": train_acc,
            "train_top_{}_acc".format(top_k): train_topk,
            "val_acc": val_acc,
            "val_top_{}_acc".format(top_k): val_topk,
        }
    F_ = train.data.shape[1]
    if kind == "linear":
        clf = LinearClassifier(F_, num_classes).to(device)
    elif kind.replace("-", "") == "nonlinear":
        clf = NonLinearClassifier(F_, num_classes).to(device)
    else:
        raise ValueError(f"unknown classifier {kind!r} (centroid | linear | nonlinear)")
    tr_acc, tr_topk, tr_loss, va_acc, va_topk, va_loss = learnable_eval(
        cfg, clf, train, val, top_k, seed=cfg["parameter"]["seed"])
    logging.info("train acc: {}, val acc: {}".format(max(tr_acc), max(va_acc)))
    return {
        "train_accuracies": tr_acc,
        "val_accuracies": va_acc,
        "train_losses": tr_loss,
        "val_losses": va_loss,
        "train_top_{}_accuracies".format(top_k): tr_topk,
        "val_top_{}_accuracies".format(top_k): va_topk,
        "lowest_val_loss": min(va_loss),
        "highest_val_acc": max(va_acc),
        "highest_val_top_k_acc": max(va_topk),
    }
