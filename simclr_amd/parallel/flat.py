"""Flat parameter store + bucketed data-parallel gradient reducer.

Reference: ``DistributedDataParallel(model, device_ids=[rank])`` with default 25 MiB buckets,
``broadcast_buffers=True`` (``/root/reference/main.py:178``): per-parameter
grads, bucket all-reduces overlapped with backward, averaged by 1/W, plus a broadcast of all BN
buffers before *every* forward.

MI355X design:

* All trainable parameters live in ONE fp32 master buffer (``master``), with a parallel fp32
  gradient buffer (``grad``), momentum buffer (owned by the optimizer) and bf16 shadow
  (``shadow``) that the compute kernels read.  Conv weights are stored OHWI (the implicit-GEMM
  K order), presented to PyTorch as OIHW-shaped ``channels_last`` views, so ``state_dict`` and
  ``nn.Module`` semantics are unchanged.  Each parameter is 64-element (256 B) aligned.
* The layout is in *reverse registration order* (≈ backward order), so gradient buckets are
  contiguous slices that fill front to back during backward.  Kernels write gradients straight
  into their slice (``ParamSlot``) and call ``mark_ready``; a full bucket is handed to RCCL on a
  dedicated comm stream (``all_reduce`` SUM; the 1/W average is folded into the LARS kernel's
  ``grad_scale``).  Buckets launch strictly in index order on every rank (RCCL requirement).
* No per-forward buffer broadcast: with SyncBN every rank already holds identical running
  statistics (the reference's per-forward broadcast is redundant traffic).
* Bucket size: default 32 MiB; on MI355X the 7 xGMI links of a GPU give the ring ~7x one link,
  so buckets of tens of MiB amortise RCCL's ~10-20 µs launch floor while the first bucket still
  starts early in the backward (``first_bucket_mb`` smaller, like DDP's 1 MiB first bucket),
  and the last one is small (``last_bucket_mb``): its all-reduce is the one left exposed after
  the backward (see ``_build_buckets``).
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

import torch
import torch.distributed as dist
from torch import nn

from ..ops.conv import ParamSlot
from . import state as pstate

ALIGN = 64


def _is_conv_weight(p: torch.Tensor) -> bool:
    return p.dim() == 4


class FlatParamStore:
    def __init__(self, model: nn.Module, device: torch.device, shadow_dtype=torch.bfloat16,
                 bucket_mb: float = 32.0, first_bucket_mb: float = 4.0,
                 last_bucket_mb: float = 2.0, group=None, world_size: Optional[int] = None, dtype=torch.float32):
        # dtype: master / gradient precision (fp32; fp64 only for the CPU equivalence tests)
        self.model = model
        self.device = torch.device(device)
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        named = list(reversed(named))  # ≈ backward order
        self.names: List[str] = [n for n, _ in named]
        self.params: List[nn.Parameter] = [p for _, p in named]
        offs, off = [], 0
        for p in self.params:
            offs.append(off)
            off += (p.numel() + ALIGN - 1) // ALIGN * ALIGN
        self.offsets = offs
        self.total = off
        self.master = torch.zeros(self.total, dtype=dtype, device=self.device)
        self.grad = torch.zeros(self.total, dtype=dtype, device=self.device)
        self.shadow = (torch.zeros(self.total, dtype=shadow_dtype, device=self.device)
                       if shadow_dtype is not None else None)
        self.slots: List[ParamSlot] = []
        for i, (p, o) in enumerate(zip(self.params, offs)):
            n = p.numel()
            src = p.detach().to(self.device, dtype)
            if _is_conv_weight(p):
                co, ci, kh, kw = p.shape
                mview = self.master[o:o + n].view(co, kh, kw, ci)
                mview.copy_(src.permute(0, 2, 3, 1))
                p.data = mview.permute(0, 3, 1, 2)
                gview = self.grad[o:o + n].view(co, kh, kw, ci)
                p.grad = gview.permute(0, 3, 1, 2)
                sview = self.shadow[o:o + n].view(co, kh, kw, ci) if self.shadow is not None else None
            else:
                mview = self.master[o:o + n].view(p.shape)
                mview.copy_(src)
                p.data = mview
                gview = self.grad[o:o + n].view(p.shape)
                p.grad = gview
                sview = self.shadow[o:o + n].view(p.shape) if self.shadow is not None else None
            slot = ParamSlot(sview, gview, i, self)
            p._slot = slot
            self.slots.append(slot)
        self.refresh_shadow()
        # ---- reducer
        st = pstate.get()
        self.group = group if group is not None else st.group
        self.world_size = world_size if world_size is not None else st.world_size
        self.comm = self.world_size > 1 or (world_size is None and group is None and st.comm)
        self._build_buckets(bucket_mb, first_bucket_mb, last_bucket_mb)
        self._comm_stream = None
        # streams that write gradients (the fused executor adds its weight-gradient stream):
        # a bucket's all-reduce waits for all of them
        self.producer_streams: List = []
        self._works: List = []
        # defer_side_join (set by the trainers, which always call finish() before reading the
        # gradients): the fused executor hands its weight-gradient stream's join to finish()
        # instead of joining at the end of its own backward, so the stem's backward (autograd,
        # after the executor) overlaps the tail of the weight gradients
        self.defer_side_join = False
        self._joins: List = []
        self.reset_step()

    # ------------------------------------------------------------------ parameters
    def refresh_shadow(self) -> None:
        """Re-derive the bf16 shadow from the fp32 master (after init / checkpoint load)."""
        if self.shadow is not None:
            with torch.no_grad():
                self.shadow.copy_(self.master)

    def rebind(self) -> None:
        """Re-point ``p.data``/``p.grad`` at the flat buffers (after load_state_dict copies)."""
        for p, slot in zip(self.params, self.slots):
            if p.grad is None or p.grad.data_ptr() != slot.grad.data_ptr():
                p.grad = slot.grad.permute(0, 3, 1, 2) if slot.grad.dim() == 4 else slot.grad

    def zero_grad(self) -> None:
        self.grad.zero_()

    def segments(self) -> List[Tuple[int, int]]:
        return [(o, p.numel()) for o, p in zip(self.offsets, self.params)]

    # ------------------------------------------------------------------ reducer
    def _build_buckets(self, bucket_mb: float, first_bucket_mb: float,
                       last_bucket_mb: float) -> None:
        """Front: one ``first_bucket_mb`` bucket (the head's gradients, ready first).  The rest
        is cut from the BACK: a small ``last_bucket_mb`` bucket (stem + layer1, the last
        gradients of the backward, whose all-reduce cannot overlap anything) and ``bucket_mb``
        buckets before it.  Cutting front-to-back instead leaves whatever remains — 16 MiB of
        layer2/layer3 gradients for ResNet-50 at 32 MiB buckets — waiting for the stem's
        gradient and then all-reduced after the backward, fully exposed."""
        mib = 1024 * 1024 / 4
        cap_first, cap = int(first_bucket_mb * mib), int(bucket_mb * mib)
        cap_last = int(last_bucket_mb * mib) if last_bucket_mb > 0 else cap
        sizes = [(p.numel() + ALIGN - 1) // ALIGN * ALIGN for p in self.params]
        P = len(sizes)
        groups: List[Tuple[int, int]] = []  # [i0, i1) param index ranges, in order
        i1, size = 0, 0
        while i1 < P and (i1 == 0 or size + sizes[i1] <= cap_first):
            size += sizes[i1]
            i1 += 1
        if i1 > 0:
            groups.append((0, i1))
        tail: List[Tuple[int, int]] = []
        end, size = P, 0
        for i in range(P - 1, i1 - 1, -1):
            limit = cap_last if not tail else cap
            if end - (i + 1) > 0 and size + sizes[i] > limit:
                tail.append((i + 1, end))
                end, size = i + 1, 0
            size += sizes[i]
        if end > i1:
            tail.append((i1, end))
        groups += reversed(tail)
        self.bucket_of: List[int] = [0] * P
        self.buckets: List[Tuple[int, int, int]] = []  # (beg, end, n_params)
        for b, (a, z) in enumerate(groups):
            for i in range(a, z):
                self.bucket_of[i] = b
            self.buckets.append((self.offsets[a], self.offsets[z] if z < P else self.total, z - a))

    def reset_step(self) -> None:
        self._ready = [0] * len(self.buckets)
        self._seen = [False] * len(self.params)
        self._next_launch = 0
        self._works = []

    def mark_ready(self, index: int) -> None:
        if not self.comm or self._seen[index]:
            return
        self._seen[index] = True
        b = self.bucket_of[index]
        self._ready[b] += 1
        while (self._next_launch < len(self.buckets)
               and self._ready[self._next_launch] == self.buckets[self._next_launch][2]):
            self._launch(self._next_launch)
            self._next_launch += 1

    def _launch(self, b: int) -> None:
        beg, end, _ = self.buckets[b]
        view = self.grad[beg:end]
        if view.is_cuda:
            if self._comm_stream is None:
                self._comm_stream = torch.cuda.Stream(device=view.device)
            cur = torch.cuda.current_stream(view.device)
            self._comm_stream.wait_stream(cur)
            for ps in self.producer_streams:
                if ps != cur:
                    self._comm_stream.wait_stream(ps)
            with torch.cuda.stream(self._comm_stream):
                work = dist.all_reduce(view, group=self.group, async_op=True)
            self._works.append(work)
        else:
            self._works.append(dist.all_reduce(view, group=self.group, async_op=True))

    def defer_join(self, stream, keep: List) -> None:
        """The compute stream joins ``stream`` in finish(); ``keep`` holds the tensors that
        stream still reads (released only after the join, so the caching allocator cannot hand
        their memory to a compute-stream allocation while they are in use)."""
        self._joins.append((stream, keep))

    def finish(self) -> None:
        """Join deferred producer streams, flush unlaunched buckets (unused params), then make
        the compute stream wait for the all-reduces."""
        if self._joins:
            cur = torch.cuda.current_stream(self.grad.device)
            for stream, keep in self._joins:
                cur.wait_stream(stream)
                keep.clear()
            self._joins = []
        if not self.comm:
            return
        while self._next_launch < len(self.buckets):
            self._launch(self._next_launch)
            self._next_launch += 1
        for w in self._works:
            w.wait()
        if self._comm_stream is not None:
            torch.cuda.current_stream(self.grad.device).wait_stream(self._comm_stream)
        self.reset_step()

    def broadcast_from(self, src: int = 0) -> None:
        """Make all ranks start from rank ``src``'s parameters and buffers (DDP ctor semantics)."""
        if not self.comm:
            return
        dist.broadcast(self.master, src=src, group=self.group)
        for b in self.model.buffers():
            dist.broadcast(b, src=src, group=self.group)
        self.refresh_shadow()
