"""LARS (Apex LARC semantics, clip=False) + SGD momentum over the flat parameter store.

Parity: ``torch.optim.SGD(exclude_from_wt_decay(...), momentum=0.9, nesterov=False,
weight_decay=0)`` wrapped in ``apex.parallel.LARC(trust_coefficient=0.001, clip=False)``
(``/root/reference/main.py:18-36,85-94``):

* wd groups by parameter *name*: any name containing ``"bias"`` or ``"bn"`` gets wd 0
  (torchvision's ``downsample.1.*`` BN params therefore DO get weight decay — replicated).
* For every parameter with a gradient: if ‖p‖ ≠ 0 and ‖g‖ ≠ 0,
  ``g ← (g + wd·p) · 0.001·‖p‖ / (‖g‖ + wd·‖p‖ + 1e-8)``; otherwise g is left untouched (no wd).
* then ``buf = m·buf + g``; ``p −= lr·buf`` (Nesterov optional for the probes).

GPU path: ``lr_step`` (closed-form schedule on device) → ``lars_norms`` (per-chunk Σp², Σg²) →
``lars_update`` (trust ratio, wd fold, momentum, fp32 master, bf16 shadow) — three launches for
the whole model, no host synchronisation, graph-capturable.  On one GPU the fused executor
issues the update of stages 4 (+ projection head), 3 and 2 from the backward as soon as their
gradients are final (``set_early_groups`` / ``early_step``, on its weight-gradient stream), so
only the layer1 + stem update trails the step.  CPU path: the same math in torch ops per
parameter (the test oracle of the kernels).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence

import torch

from ..ops import registry
from ..parallel.flat import FlatParamStore
from .schedule import MODE_WARMUP_COSINE, lr_at

CHUNK = 16384


def exclude_from_wt_decay(named_params, weight_decay: float, skip_list=("bias", "bn")):
    """Reference param-group rule (main.py:18-36), returned as torch-style groups."""
    params, excluded = [], []
    for name, param in named_params:
        if not param.requires_grad:
            continue
        if any(layer_name in name for layer_name in skip_list):
            excluded.append(param)
        else:
            params.append(param)
    return [{"params": params, "weight_decay": weight_decay},
            {"params": excluded, "weight_decay": 0.0}]


def weight_decay_per_param(store: FlatParamStore, weight_decay: float,
                           skip_list: Optional[Sequence[str]] = ("bias", "bn")) -> List[float]:
    out = []
    for name in store.names:
        if skip_list is not None and any(s in name for s in skip_list):
            out.append(0.0)
        else:
            out.append(weight_decay)
    return out


class _ChunkTable:
    """Chunk tables of the LARS kernels over a subset of the store's parameters: chunks in
    segment order; per-segment chunk ranges index this table (0, 0 outside the subset)."""

    def __init__(self, store: FlatParamStore, idx: Sequence[int], dev):
        segs = store.segments()
        cseg, cbeg, cend = [], [], []
        sbeg, send = [0] * len(segs), [0] * len(segs)
        for i in idx:
            o, n = segs[i]
            sbeg[i] = len(cseg)
            for b in range(o, o + n, CHUNK):
                cseg.append(i)
                cbeg.append(b)
                cend.append(min(b + CHUNK, o + n))
            send[i] = len(cseg)
        i32 = dict(device=dev, dtype=torch.int32)
        self.nchunks = len(cseg)
        self.seg = torch.tensor(cseg, **i32)
        self.beg = torch.tensor(cbeg, **i32)
        self.end = torch.tensor(cend, **i32)
        self.seg_beg = torch.tensor(sbeg, **i32)
        self.seg_end = torch.tensor(send, **i32)
        self.norms = torch.zeros(max(1, 2 * len(cseg)), device=dev, dtype=torch.float32)


class FusedLARS:
    def __init__(self, store: FlatParamStore, weight_decays: Sequence[float], lr0: float,
                 momentum: float = 0.9, nesterov: bool = False, trust_coefficient: float = 0.001,
                 eps: float = 1e-8, lars: bool = True, schedule_mode: int = MODE_WARMUP_COSINE,
                 warmup_steps: int = 0, total_steps: int = 0, start_step: int = 0,
                 grad_scale: Optional[float] = None):
        self.store = store
        dev = store.device
        self.lr0 = float(lr0)
        self.momentum = float(momentum)
        self.nesterov = bool(nesterov)
        self.trust = float(trust_coefficient)
        self.eps = float(eps)
        self.lars = bool(lars)
        self.mode = int(schedule_mode)
        self.warmup = int(warmup_steps)
        self.total = int(total_steps)
        self.grad_scale = float(grad_scale if grad_scale is not None else 1.0 / store.world_size)
        assert len(weight_decays) == len(store.params)
        self.weight_decays = [float(w) for w in weight_decays]
        cseg, cbeg, cend, sbeg, send = [], [], [], [], []
        for i, (o, n) in enumerate(store.segments()):
            sbeg.append(len(cseg))
            for b in range(o, o + n, CHUNK):
                cseg.append(i)
                cbeg.append(b)
                cend.append(min(b + CHUNK, o + n))
            send.append(len(cseg))
        i32 = dict(device=dev, dtype=torch.int32)
        self._groups: Dict[int, _ChunkTable] = {}  # early-update groups (set_early_groups)
        self._rest: Optional[_ChunkTable] = None
        self._issued: set = set()
        self.early_issued = 0  # groups issued through early_step (tests / accounting)
        self.chunk_seg = torch.tensor(cseg, **i32)
        self.chunk_beg = torch.tensor(cbeg, **i32)
        self.chunk_end = torch.tensor(cend, **i32)
        self.seg_chunk_beg = torch.tensor(sbeg, **i32)
        self.seg_chunk_end = torch.tensor(send, **i32)
        self.seg_wd = torch.tensor(self.weight_decays, device=dev, dtype=torch.float32)
        flags = [(1 if self.lars else 0) | (2 if store.shadow is not None else 0)
                 for _ in store.params]
        self.seg_flags = torch.tensor(flags, **i32)
        self.norms = torch.zeros(2 * len(cseg), device=dev, dtype=torch.float32)
        self.mom = torch.zeros(store.total, device=dev, dtype=torch.float32)
        self.step_t = torch.tensor([int(start_step)], device=dev, dtype=torch.int64)
        self.lr_t = torch.zeros(1, device=dev, dtype=torch.float32)
        self.host_step = int(start_step)

    # -------------------------------------------------------------- API
    @property
    def last_lr(self) -> float:
        """LR used by the most recent step (computed on host from the step count: no sync)."""
        return lr_at(self.mode, max(self.host_step - 1, 0), self.lr0, self.warmup, self.total)

    @property
    def logged_lr(self) -> float:
        """``optimizer.param_groups[0]["lr"]`` as the reference reads it after a step: the
        cosine scheduler has already advanced past warmup (main.py:119-127)."""
        s = max(self.host_step - 1, 0)
        if self.mode == MODE_WARMUP_COSINE and s <= self.warmup:
            return lr_at(self.mode, s, self.lr0, self.warmup, self.total)
        return lr_at(self.mode, s + 1, self.lr0, self.warmup, self.total)

    @property
    def param_groups(self):
        return [{"lr": self.logged_lr}]

    def zero_grad(self, set_to_none: bool = False) -> None:
        self.store.zero_grad()

    def set_early_groups(self, groups: Dict[int, Sequence[int]]) -> None:
        """Parameter groups (``key`` → indices into ``store.params``) whose update the backward
        may issue before ``step()`` with ``early_step(key)``, once their gradients are final
        (the fused executor does so per stage, on its weight-gradient stream, so the update
        overlaps the rest of the backward instead of trailing it); ``step()`` then updates the
        groups not issued early and every other parameter.  Same kernels, chunk order and
        per-segment reduction as the single update: the result is bitwise identical."""
        dev = self.store.device
        covered = set()
        self._groups = {}
        for key, idx in groups.items():
            self._groups[int(key)] = _ChunkTable(self.store, sorted(idx), dev)
            covered |= set(idx)
        self._rest = _ChunkTable(self.store, [i for i in range(len(self.store.params))
                                              if i not in covered], dev)
        self._issued = set()

    def _hip(self) -> bool:
        m = self.store.master
        return m.is_cuda and registry.use_hip(m)

    def _launch(self, ops, t: "_ChunkTable") -> None:
        if t.nchunks == 0:
            return
        m = self.store.master
        ops.lars_norms(m, self.store.grad, t.beg, t.end, self.grad_scale, t.norms)
        ops.lars_update(m, self.store.grad, self.mom, self.store.shadow, t.seg, t.beg, t.end,
                        t.seg_beg, t.seg_end, self.seg_wd, self.seg_flags, t.norms, self.lr_t,
                        self.momentum, self.trust, self.eps, self.grad_scale, self.nesterov)

    def _lr_step(self, ops) -> None:
        ops.lr_step(self.step_t, self.lr_t, self.lr0, self.warmup, self.total, self.mode)

    def early_step(self, key: int) -> None:
        """Issue group ``key``'s update now, on the current stream (see set_early_groups)."""
        if key not in self._groups or key in self._issued or not self._hip():
            return
        ops = torch.ops.simclr_amd
        if not self._issued:
            self._lr_step(ops)
        self._issued.add(key)
        self.early_issued += 1
        self._launch(ops, self._groups[key])

    def step(self) -> None:
        m = self.store.master
        if m.is_cuda and registry.use_hip(m):
            ops = torch.ops.simclr_amd
            if self._rest is None:
                self._lr_step(ops)
                ops.lars_norms(m, self.store.grad, self.chunk_beg, self.chunk_end,
                               self.grad_scale, self.norms)
                ops.lars_update(m, self.store.grad, self.mom, self.store.shadow, self.chunk_seg,
                                self.chunk_beg, self.chunk_end, self.seg_chunk_beg,
                                self.seg_chunk_end, self.seg_wd, self.seg_flags, self.norms,
                                self.lr_t, self.momentum, self.trust, self.eps,
                                self.grad_scale, self.nesterov)
            else:
                if not self._issued:
                    self._lr_step(ops)
                for key, t in self._groups.items():
                    if key not in self._issued:
                        self._launch(ops, t)
                self._launch(ops, self._rest)
                self._issued = set()
        else:
            self._step_torch()
        self.host_step += 1

    @torch.no_grad()
    def _step_torch(self) -> None:
        s = int(self.step_t.item())
        lr = lr_at(self.mode, s, self.lr0, self.warmup, self.total)
        self.step_t.fill_(s + 1)
        self.lr_t.fill_(lr)
        st = self.store
        for (o, n), wd in zip(st.segments(), self.weight_decays):
            p = st.master[o:o + n]
            g = st.grad[o:o + n] * self.grad_scale
            buf = self.mom[o:o + n]
            if self.lars:
                pn = torch.norm(p)
                gn = torch.norm(g)
                if pn != 0 and gn != 0:
                    local = self.trust * pn / (gn + pn * wd + self.eps)
                    d = (g + wd * p) * local
                else:
                    d = g
            else:
                d = g + wd * p
            buf.mul_(self.momentum).add_(d)
            upd = d + self.momentum * buf if self.nesterov else buf
            p.sub_(lr * upd)
        st.refresh_shadow()

    def state_dict(self) -> dict:
        return {"mom": self.mom.detach().cpu(), "step": int(self.host_step)}

    def load_state_dict(self, sd: dict) -> None:
        self.mom.copy_(sd["mom"].to(self.mom.device))
        self.host_step = int(sd["step"])
        self.step_t.fill_(self.host_step)
