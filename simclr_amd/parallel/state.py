"""Process-global parallel state (rank / world / process group) used by the ops.

The reference binds the rank from the Hydra override ``distributed.local_rank`` and passes it
as the *global* rank to ``init_process_group`` (``/root/reference/distributed_utils.py:8-20``),
which breaks multi-node.  Here the global rank always comes from the ``RANK`` /
``WORLD_SIZE`` environment written by the launcher or torchrun; ``LOCAL_RANK`` picks the GPU.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class ParallelState:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    group: Optional[object] = None
    backend: str = "none"
    # second communicator for the latency-critical BatchNorm statistics all-reduces, so they
    # never queue behind a multi-MiB gradient-bucket all-reduce on the same RCCL stream
    stat_group: Optional[object] = None
    # third communicator for the downsample branch's BN statistics (it runs on its own stream,
    # concurrently with the main branch: sharing a communicator would order their all-reduces)
    branch_stat_group: Optional[object] = None
    # run every collective even at world_size 1 (a 1-rank RCCL group): exercises the
    # multi-GPU code path (comm streams, async handles, the stats communicator) on one GPU
    force_comm: bool = False
    # one-shot IPC exchange of BatchNorm statistics (comm/ipc.py), replacing the statistics
    # all-reduces at world > 1 when its self-test passed on every rank
    ipc: Optional[object] = None

    @property
    def stats_group(self):
        return self.stat_group if self.stat_group is not None else self.group

    @property
    def distributed(self) -> bool:
        return self.world_size > 1

    @property
    def comm(self) -> bool:
        """True when the step issues collectives (multi-rank, or ``force_comm``)."""
        return self.world_size > 1 or (self.force_comm and self.group is not None)


_STATE = ParallelState()


def get() -> ParallelState:
    return _STATE


def set_state(**kw) -> ParallelState:
    for k, v in kw.items():
        setattr(_STATE, k, v)
    return _STATE


def make_stat_group(st: "ParallelState") -> None:
    """Create the BN-statistics communicator (collective call: every rank, same order)."""
    if st.comm and st.stat_group is None and dist.is_initialized():
        st.stat_group = dist.new_group(list(range(st.world_size)))
        st.branch_stat_group = dist.new_group(list(range(st.world_size)))


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


def tag_sites(model: torch.nn.Module) -> None:
    """Name every BatchNorm of ``model`` after its qualified module name (the IPC site key)."""
    for name, m in model.named_modules():
        if hasattr(m, "running_mean") and hasattr(m, "num_features"):  # ours and torch's BN
            m._site_name = name


def site_key(bn: torch.nn.Module, direction: str):
    """Stable exchange-site key of a BatchNorm (``tag_sites``; an untagged module falls back
    to its object identity)."""
    name = bn.__dict__.get("_site_name")
    if name is None:
        name = f"untagged-{type(bn).__name__}-{id(bn)}"
    return (name, direction)
