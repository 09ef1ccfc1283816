"""Process-global parallel state (rank / world / process group) used by the ops.

The reference binds the rank from the Hydra override ``distributed.local_rank`` and passes it
as the *global* rank to ``init_process_group`` (``/root/reference/distributed_utils.py:8-20``),
which breaks multi-node.  Here the global rank always comes from the ``RANK`` /
``WORLD_SIZE`` environment written by the launcher or torchrun; ``LOCAL_RANK`` picks the GPU.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch.distributed as dist


@dataclass
class ParallelState:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    group: Optional[object] = None
    backend: str = "none"

    @property
    def distributed(self) -> bool:
        return self.world_size > 1


_STATE = ParallelState()


def get() -> ParallelState:
    return _STATE


def set_state(**kw) -> ParallelState:
    for k, v in kw.items():
        setattr(_STATE, k, v)
    return _STATE


def reset() -> None:
    global _STATE
    _STATE = ParallelState()


def world_size() -> int:
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(_STATE.group)
    return 1


def rank() -> int:
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(_STATE.group)
    return 0
