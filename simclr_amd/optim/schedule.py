"""Learning-rate scaling and schedule.

Parity: ``calculate_initial_lr`` / ``calculate_lr`` (``/root/reference/lr_utils.py:5-26``) and the
warmup-then-``CosineAnnealingLR`` sequencing of ``/root/reference/main.py:73-80,96-122``.
SURVEY C19 derives the closed form the reference's recursive scheduler produces:

    lr(s) = s / W · lr0                                   for s ≤ W   (lr0 if W == 0)
    lr(s) = lr0 · ½ (1 + cos(π (s − W − 1) / (T − W)))    for s > W

(steps W and W+1 both run at lr0, step 0 at 0).  ``lr0 = lr · batches / 256`` with the *per-GPU*
batch, or ``lr · sqrt(batches)`` without ``linear_schedule``.  The GPU path
evaluates the same closed form on device (``csrc/lars.hip: k_lr_step``) so the optimizer step
needs no host round trip.
"""
from __future__ import annotations

import math


def _get(cfg, a, b):
    return cfg[a][b]


def calculate_initial_lr(cfg) -> float:
    if _get(cfg, "parameter", "linear_schedule"):
        return _get(cfg, "experiment", "lr") * _get(cfg, "experiment", "batches") / 256.0
    return _get(cfg, "experiment", "lr") * math.sqrt(_get(cfg, "experiment", "batches"))


def calculate_lr(cfg, warmup_steps: int, current_steps: int) -> float:
    initial_lr = calculate_initial_lr(cfg)
    if warmup_steps > 0.0:
        return current_steps / warmup_steps * initial_lr
    return initial_lr


def warmup_cosine_lr(step: int, lr0: float, warmup: int, total: int) -> float:
    """Closed form of the reference schedule at optimizer step ``step`` (0-based)."""
    if step <= warmup:
        return step / warmup * lr0 if warmup > 0 else lr0
    T = total - warmup
    if T <= 0:
        return lr0
    return lr0 * 0.5 * (1.0 + math.cos(math.pi * (step - warmup - 1) / T))


def cosine_lr(step: int, lr0: float, total: int) -> float:
    """``CosineAnnealingLR(T_max=total)`` stepped after every batch from step 0 (linear probe,
    ``/root/reference/eval.py:148-163``)."""
    if total <= 0:
        return lr0
    return lr0 * 0.5 * (1.0 + math.cos(math.pi * step / total))


MODE_WARMUP_COSINE = 0
MODE_COSINE = 1
MODE_CONSTANT = 2


def lr_at(mode: int, step: int, lr0: float, warmup: int, total: int) -> float:
    if mode == MODE_WARMUP_COSINE:
        return warmup_cosine_lr(step, lr0, warmup, total)
    if mode == MODE_COSINE:
        return cosine_lr(step, lr0, total)
    return lr0
