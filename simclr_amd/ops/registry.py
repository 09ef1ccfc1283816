"""Single dispatch point between the hand-written HIP kernels and the torch-op oracles.

Rules (no silent fallbacks on the GPU):

* CPU tensors always take the torch-op path (that is the numerics oracle and the gloo /
  CPU-test path).
* CUDA (= HIP on ROCm) tensors take the HIP kernels of ``simclr_amd/_C`` unless the user asked
  for ``backend=torch`` explicitly (used to measure the reference-semantics baseline).  If the
  extension is missing on a GPU box the op raises instead of quietly running torch ops.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn.functional as F

from ..parallel import state as pstate

_BACKEND = os.environ.get("SIMCLR_BACKEND", "auto")
_VALID = ("auto", "hip", "torch")


def set_backend(name: str) -> None:
    global _BACKEND
    if name not in _VALID:
        raise ValueError(f"backend must be one of {_VALID}, got {name!r}")
    _BACKEND = name


def get_backend() -> str:
    return _BACKEND


def use_hip(t: torch.Tensor) -> bool:
    if not t.is_cuda or _BACKEND == "torch":
        return False
    from . import _ext
    _ext.require()
    return True


# --------------------------------------------------------------------------- batch norm
def batch_norm_train(x, bn, segments: int = 1, residual: Optional[torch.Tensor] = None,
                     relu: bool = False):
    st = pstate.get()
    if x.dtype == torch.bfloat16 and use_hip(x):
        from . import batchnorm_hip
        return batchnorm_hip.batch_norm_train(x, bn, segments, residual, relu, st)
    from .batchnorm import reference_batch_norm_train
    return reference_batch_norm_train(x, bn, segments, residual, relu,
                                      group=st.group, world_size=st.world_size)


def batch_norm_eval(x, bn, residual: Optional[torch.Tensor] = None, relu: bool = False):
    if x.dtype == torch.bfloat16 and use_hip(x):
        from . import batchnorm_hip
        return batchnorm_hip.batch_norm_eval(x, bn, residual, relu)
    from .batchnorm import reference_batch_norm_eval
    return reference_batch_norm_eval(x, bn, residual, relu)
