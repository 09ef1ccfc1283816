"""Checkpoint I/O in the reference's format, plus resumable training state.

Reference contract (``/root/reference/main.py:129-131``): rank 0 writes
``torch.save(ddp_model.state_dict(), "epoch={E}-{output_model_name}")`` — an ``OrderedDict`` of
fp32 NCHW/OIHW tensors with torchvision names and the DDP ``module.`` prefix (weights + BN
buffers only).  Readers strip ``module.`` (eval.py:257) and load ``strict=False``.

This module writes exactly that (contiguous fp32 CPU tensors, regardless of the internal OHWI /
flat-buffer layout), and additionally a ``resume-<E>.pt`` with optimizer momentum, step, epoch
and RNG state (an extension: the reference cannot resume).  Loading always uses
``torch.load(..., weights_only=True)``.
"""
from __future__ import annotations

from collections import OrderedDict
from pathlib import Path
from typing import Optional

import torch
from torch import nn

PREFIX = "module."


def reference_state_dict(model: nn.Module, prefix: str = PREFIX) -> "OrderedDict[str, torch.Tensor]":
    out = OrderedDict()
    for k, v in model.state_dict().items():
        t = v.detach()
        if t.is_floating_point():
            t = t.float()
        out[prefix + k] = t.contiguous().cpu().clone()
    return out


def save_reference_checkpoint(model: nn.Module, path: str) -> None:
    torch.save(reference_state_dict(model), path)


def checkpoint_name(epoch: int, output_model_name: str) -> str:
    return "epoch={}-{}".format(epoch, output_model_name)


def strip_prefix(sd: dict, prefix: str = PREFIX) -> dict:
    return {(k[len(prefix):] if k.startswith(prefix) else k): v for k, v in sd.items()}


def load_state(path, map_location="cpu") -> dict:
    return torch.load(path, map_location=map_location, weights_only=True)


@torch.no_grad()
def load_into(model: nn.Module, path, strict: bool = False, store=None):
    """Load a reference-format checkpoint (prefix stripped) into ``model`` in place, keeping the
    flat-store views intact (copy_ into existing tensors, never rebind)."""
    sd = strip_prefix(load_state(path))
    own = model.state_dict(keep_vars=True)
    missing, unexpected = [], []
    for k, v in sd.items():
        if k not in own:
            unexpected.append(k)
            continue
        tgt = own[k]
        tgt.data.copy_(v.to(tgt.device, tgt.dtype).reshape(tgt.shape))
    for k in own:
        if k not in sd:
            missing.append(k)
    if strict and (missing or unexpected):
        raise RuntimeError(f"state_dict mismatch: missing={missing} unexpected={unexpected}")
    if store is not None:
        store.refresh_shadow()
    return missing, unexpected


def _local_rng() -> dict:
    """This process's generators: host torch, its OWN device's CUDA generator, NumPy."""
    cuda = None
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        cuda = torch.cuda.get_rng_state()
    return {"torch_rng": torch.get_rng_state(), "cuda_rng_device": cuda,
            "numpy_rng": _numpy_rng_state()}


def gather_rng_states(dst: int = 0, group=None) -> Optional[list]:
    """Collective: every rank's ``_local_rng()``, as a rank-indexed list on ``dst`` (None on
    the other ranks).  Call it on every rank when rank ``dst`` saves a resume file."""
    import torch.distributed as dist
    mine = _local_rng()
    if group is None or not dist.is_initialized():
        return [mine]
    world = dist.get_world_size(group)
    out = [None] * world if dist.get_rank(group) == dst else None
    dist.gather_object(mine, out, dst=dst, group=group)
    return out


def save_resume(path: str, model: nn.Module, optimizer, epoch: int, step: int,
                extra: Optional[dict] = None, group=None) -> None:
    """Resume file (rank 0 writes it).  ``group``: multi-rank job — every other rank must call
    ``gather_rng_states(0, group)`` at the same point, so the file holds each rank's own
    generators (``rank_rng[r]``), restored per rank by ``restore_rng``."""
    local = _local_rng()
    ranks = gather_rng_states(0, group) if group is not None else [local]
    torch.save({
        "model": reference_state_dict(model),
        "optimizer": optimizer.state_dict() if optimizer is not None else None,
        "epoch": int(epoch),
        "step": int(step),
        "torch_rng": local["torch_rng"],
        "numpy_rng": local["numpy_rng"],
        "rank_rng": ranks,
        "extra": extra or {},
    }, path)


def _numpy_rng_state() -> dict:
    """NumPy's global MT19937 state as tensors / ints (loadable with ``weights_only=True``)."""
    import numpy as np
    name, keys, pos, has_gauss, gauss = np.random.get_state()
    return {"keys": torch.from_numpy(keys.astype(np.int64)), "pos": int(pos),
            "has_gauss": int(has_gauss), "gauss": float(gauss)}


def restore_rng(blob: dict, rank: Optional[int] = None) -> None:
    """Restore this rank's host / device / NumPy generators saved by ``save_resume``: the
    ``rank_rng[rank]`` entry (each rank gets its own state back, its device generator on its
    current device); files without one fall back to the top-level host / NumPy state."""
    import numpy as np
    import torch.distributed as dist
    if rank is None:
        rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
    ranks = blob.get("rank_rng") or []
    ent = ranks[rank] if rank < len(ranks) else blob
    if ent.get("torch_rng") is not None:
        torch.set_rng_state(ent["torch_rng"])
    cuda = ent.get("cuda_rng_device")
    if cuda is None and torch.cuda.is_available():
        # resume files written before the per-rank entries: one device state per GPU, top level
        legacy = blob.get("cuda_rng")
        dev = torch.cuda.current_device()
        if isinstance(legacy, (list, tuple)) and dev < len(legacy):
            cuda = legacy[dev]
        else:
            import logging
            logging.getLogger(__name__).warning(
                "resume file holds no device RNG state for rank %d: the GPU augmentation stream "
                "is NOT restored (it restarts from the seed)", rank)
    if cuda is not None and torch.cuda.is_available():
        torch.cuda.set_rng_state(cuda)
    n = ent.get("numpy_rng")
    if n:
        np.random.set_state(("MT19937", n["keys"].numpy().astype(np.uint32), n["pos"],
                             n["has_gauss"], n["gauss"]))


def load_resume(path, model: nn.Module, optimizer=None, store=None) -> dict:
    blob = torch.load(path, map_location="cpu", weights_only=True)
    own = model.state_dict(keep_vars=True)
    with torch.no_grad():
        for k, v in strip_prefix(blob["model"]).items():
            if k in own:
                own[k].data.copy_(v.to(own[k].device, own[k].dtype).reshape(own[k].shape))
    if store is not None:
        store.refresh_shadow()
    if optimizer is not None and blob.get("optimizer") is not None:
        optimizer.load_state_dict(blob["optimizer"])
    restore_rng(blob)
    return blob
