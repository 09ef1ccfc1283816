"""Per-shape kernel-variant autotuning (tile shape of the implicit-GEMM kernels).

The first time a problem shape is seen in eager mode every admissible tile variant is timed
with HIP events on an otherwise idle device (3 launches after 1 warm-up, best of
``SIMCLR_AUTOTUNE_ROUNDS`` = 2 sweeps) and the fastest is cached for the process; inside a
hipGraph capture, or with ``SIMCLR_AUTOTUNE=0``, the cached (else default) variant is used.
Tuning launches write only to scratch outputs, so it has no side effects.
"""
from __future__ import annotations

import os
from typing import Callable, Dict, Hashable, Sequence

import torch

_CACHE: Dict[Hashable, int] = {}
ENABLED = os.environ.get("SIMCLR_AUTOTUNE", "1") != "0"
ROUNDS = int(os.environ.get("SIMCLR_AUTOTUNE_ROUNDS", "2"))


def set_enabled(on: bool) -> None:
    """``runtime.deterministic`` turns tuning off: timing-driven choices differ run to run, and
    with them the fp32 summation order of a kernel (bitwise reproducibility needs fixed tiles)."""
    global ENABLED
    if bool(on) != ENABLED:
        _CACHE.clear()  # choices made under the other policy (timed vs fixed) must not leak
    ENABLED = bool(on)


def cached(key: Hashable):
    return _CACHE.get(key)


def pick(key: Hashable, candidates: Sequence[int], default: int,
         run: Callable[[int], None], reps: int = 3) -> int:
    if key in _CACHE:
        return _CACHE[key]
    cands = list(candidates)
    if not cands:
        return default
    if (not ENABLED or len(cands) == 1 or not torch.cuda.is_available()
            or torch.cuda.is_current_stream_capturing()):
        choice = default if default in cands else cands[0]
        if not (torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()):
            _CACHE[key] = choice  # fixed choice: later launches skip the candidate walk
        return choice
    # Trials run with the device otherwise idle (the step's side streams — weight gradients,
    # downsample branch, gradient all-reduce — would share the CUs with whichever candidate
    # happened to be timed under them) and each candidate keeps the best of ROUNDS sweeps: with
    # one sweep on a busy device the choice for ~40 % of the shapes changed from run to run,
    # some by 15-20 % in kernel time.
    torch.cuda.synchronize()
    best_t = {v: float("inf") for v in cands}
    for _ in range(ROUNDS):
        for v in cands:
            run(v)
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(reps):
                run(v)
            e.record()
            e.synchronize()
            best_t[v] = min(best_t[v], s.elapsed_time(e))
    best = min(cands, key=lambda v: (best_t[v], cands.index(v)))
    _CACHE[key] = best
    return best


def table() -> Dict[Hashable, int]:
    return dict(_CACHE)


def sync_from_rank0(group=None) -> int:
    """Adopt rank 0's choices on every rank (collective; call it on all ranks after the eager
    steps that tuned).  Each rank times its candidates on its own GPU, so near-ties can resolve
    differently and the ranks would run different tiles — different fp32 summation orders —
    where the reference pins one algorithm everywhere (``cudnn.deterministic=True,
    benchmark=False``, /root/reference/main.py:150-151).  Returns the number of entries this
    rank changed."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) < 2:
        return 0
    obj = [dict(_CACHE) if dist.get_rank(group) == 0 else None]
    dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None
                               else 0, group=group)
    theirs = obj[0] or {}
    changed = sum(1 for k, v in theirs.items() if _CACHE.get(k) != v)
    _CACHE.update(theirs)
    return changed
