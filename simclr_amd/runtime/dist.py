"""Process-group bootstrap and device binding.

Reference: ``init_ddp`` (``/root/reference/distributed_utils.py:8-20``) — NCCL, ``env://``
rendezvous, ``rank = cfg.distributed.local_rank`` (wrong across nodes), then
``torch.cuda.set_device(rank)``; ``cleanup()`` is never called.

Here: the *global* rank / world size come from ``RANK`` / ``WORLD_SIZE`` (written by our
launcher and by torchrun), the GPU from ``LOCAL_RANK``; without those variables the run is single-process (the
Hydra keys ``distributed.local_rank`` / ``distributed.world_size`` that launch.py still appends
for command-line compatibility must agree with the environment).  Backend: ``nccl`` (= RCCL over xGMI on ROCm) on GPUs, ``gloo``
on CPU.  A process-group timeout makes a dead peer an error instead of a hang.
"""
from __future__ import annotations

import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist

from ..parallel import state as pstate


def resolve_world(cfg=None):
    env = os.environ
    if "WORLD_SIZE" in env and "RANK" in env:
        world = int(env["WORLD_SIZE"])
        rank = int(env["RANK"])
        local = int(env.get("LOCAL_RANK", rank))
        return rank, world, local
    # Without RANK/WORLD_SIZE (not launched by launch.py / torchrun) run single-process: the
    # reference's default ``distributed.world_size=4`` would otherwise wait forever for peers.
    return 0, 1, 0


def pick_device(local_rank: int, use_cuda: bool = True) -> torch.device:
    if use_cuda and torch.cuda.is_available():
        torch.cuda.set_device(local_rank % torch.cuda.device_count())
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


# process-group timeout: a rank that dies or hangs fails every collective of its peers within
# this bound (the fail-fast launcher then stops the job) instead of holding the node for
# torch's default 30 minutes; ``runtime.pg_timeout_s`` overrides it
DEFAULT_PG_TIMEOUT_S = 600.0


def init_distributed(cfg=None, use_cuda: bool = True, backend: Optional[str] = None,
                     timeout_s: Optional[float] = None) -> pstate.ParallelState:
    rank, world, local = resolve_world(cfg)
    if timeout_s is None:
        rt = (cfg or {}).get("runtime", {}) if hasattr(cfg or {}, "get") else {}
        timeout_s = float((rt or {}).get("pg_timeout_s", None) or DEFAULT_PG_TIMEOUT_S)
    device = pick_device(local, use_cuda)
    if world > 1 and not dist.is_initialized():
        be = backend or ("nccl" if device.type == "cuda" else "gloo")
        url = "env://"
        if cfg is not None and "distributed" in cfg:
            url = cfg["distributed"].get("dist_url", "env://") or "env://"
        kw = dict(backend=be, init_method=url, world_size=world, rank=rank,
                  timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = device
        try:
            dist.init_process_group(**kw)
        except TypeError:
            kw.pop("device_id", None)
            dist.init_process_group(**kw)
    st = pstate.set_state(rank=rank, world_size=world, local_rank=local,
                          group=dist.group.WORLD if world > 1 else None,
                          backend=(dist.get_backend() if world > 1 else "none"))
    st.device = device
    pstate.make_stat_group(st)
    if st.comm and device.type == "cuda":
        # BatchNorm statistics over IPC-mapped peer memory (self-tested; RCCL otherwise)
        from ..comm import setup_stats_exchange
        setup_stats_exchange(st, device)
    return st


def cleanup() -> None:
    ipc = getattr(pstate.get(), "ipc", None)
    if ipc is not None:
        if dist.is_available() and dist.is_initialized():
            dist.barrier()  # no peer still reads this rank's arena through its mapping
        ipc.close()
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()
    pstate.reset()


def barrier() -> None:
    st = pstate.get()
    if st.world_size > 1:
        dist.barrier(group=st.group)
