"""Small shared helpers: config access with defaults, seeding, JSONL metrics."""
from __future__ import annotations

import json
import os
import random
import time
from typing import Any, Optional

import numpy as np
import torch


def cfg_get(cfg, dotted: str, default: Any = None) -> Any:
    cur = cfg
    for part in dotted.split("."):
        if isinstance(cur, dict) and part in cur:
            cur = cur[part]
        else:
            return default
    return default if cur is None and default is not None else cur


def seed_everything(seed: int, deterministic: bool = False) -> None:
    """Reference seeding (main.py:146-151): numpy + torch + all GPUs, same seed on every rank.

    The reference also sets ``cudnn.deterministic = True``; on ROCm that flag selects MIOpen's
    deterministic convolution solvers, which run the stock-op (``runtime.backend=torch``)
    ResNet-18 step in 12.2 s instead of 85 ms (tools/torch_step_probe.py on MI355X), so it is set
    only with ``runtime.deterministic=true``.  The HIP kernels never use MIOpen; their
    determinism switch is the fixed-tile policy (``ops.tuning.set_enabled(False)``)."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    torch.backends.cudnn.benchmark = False
    torch.backends.cudnn.deterministic = bool(deterministic)
    if deterministic:
        torch.use_deterministic_algorithms(True, warn_only=True)


class MetricsWriter:
    """Append-only JSONL metrics stream (epoch, step, loss, lr, images/sec, ...)."""

    def __init__(self, path: Optional[str]):
        self.f = open(path, "a") if path else None

    def write(self, **kw) -> None:
        if self.f is None:
            return
        kw.setdefault("time", time.time())
        self.f.write(json.dumps(kw) + "\n")
        self.f.flush()

    def close(self) -> None:
        if self.f is not None:
            self.f.close()
            self.f = None


# attribution knobs that change the math (bench / tools only): a leftover export in a training
# shell would silently train a wrong model
EXPERIMENT_KNOBS = ("SIMCLR_SKIP_WGRAD", "SIMCLR_EXPERIMENT_WGRAD_SLABS",
                    "SIMCLR_EXPERIMENT_SKIP_BNREDUCE")


def refuse_experiment_knobs(where: str) -> None:
    import os
    bad = [k for k in EXPERIMENT_KNOBS if os.environ.get(k, "0") not in ("", "0")]
    if bad:
        raise RuntimeError(f"{where}: {', '.join(bad)} set — these attribution experiments drop "
                           "weight gradients / BatchNorm statistics and are refused outside "
                           "bench.py and tools/")
