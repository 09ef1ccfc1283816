"""NT-Xent loss (normalised temperature-scaled cross entropy).

Reference API: ``NT_Xent(temperature, reduction, device)(view0, view1)``
(``/root/reference/loss.py:4-65``).  Semantics: anchors are the 2N rows of both
views; for each, the logits are cosine similarities / τ to every other row (self excluded), the
target is the same image's other view; ``reduction="mean"`` averages over the 2N anchors,
``"sum"`` sums, ``"none"`` returns a (2, N) tensor [view0 anchors; view1 anchors].

Extension (north star): ``gather=True`` all-gathers the bf16 embeddings z of every
rank over RCCL on a side stream, overlapped with this rank's normalisation and the scoring of
its own columns (the peers' columns are scored into further online-LSE partials once they
arrive), so each anchor sees 2·N·W − 1 candidates instead of 2N − 1 (negatives from the global
batch).  The gradient w.r.t. the gathered columns returns through a reduce-scatter on a side
stream, overlapped with the row-gradient kernel.
Parity default is ``gather=False`` (the reference's loss is per-GPU local).

GPU path: the fused exact-fp32 MFMA kernels of ``csrc/ntxent.hip`` (no N×N logits, no mask or
concat copies, no host→device target upload per call).  CPU / fp32 path: torch ops.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch import nn

from ..ops import registry
from ..parallel import state as pstate


def nt_xent_torch(z: torch.Tensor, n: int, temperature: float, reduction: str = "mean",
                  gather: bool = False, group=None, world_size: int = 1, rank: int = 0):
    """Oracle implementation on torch ops; ``z`` = [view0; view1] of shape [2n, d]."""
    zn = F.normalize(z if z.dtype == torch.float64 else z.float(), p=2, dim=1)
    R = zn.shape[0]
    if gather and world_size > 1:
        from torch.distributed.nn.functional import all_gather
        cols = torch.cat(all_gather(zn, group=group), dim=0)
        col_offset = rank * R
    else:
        cols = zn
        col_offset = 0
    sim = zn @ cols.t() / temperature
    idx = torch.arange(R, device=z.device)
    self_mask = torch.zeros_like(sim, dtype=torch.bool)
    self_mask[idx, col_offset + idx] = True
    sim = sim.masked_fill(self_mask, float("-inf"))
    targets = col_offset + torch.where(idx < n, idx + n, idx - n)
    rows = F.cross_entropy(sim, targets, reduction="none")
    if reduction == "none":
        return rows.view(2, n)
    if reduction == "sum":
        return rows.sum()
    return rows.sum() / n * 0.5


_SIDE: dict = {}


def _side_stream(dev: torch.device) -> "torch.cuda.Stream":
    """Per-device side stream of the gathered loss's collectives."""
    if dev not in _SIDE:
        _SIDE[dev] = torch.cuda.Stream(device=dev)
    return _SIDE[dev]


# z all-gathers the fused projection head already issued on the side stream, one per view, each
# under the next view's GEMM 2 (models/head_fused.py): (device, z.data_ptr()) -> (zb_all,
# tensors the side stream still uses).  The loss takes the gathered rows from here instead of
# issuing its own all-gather.
_PREGATHER: dict = {}


def register_pregather(z: torch.Tensor, zb_all: torch.Tensor, keep) -> None:
    _PREGATHER.clear()  # one step in flight per process
    _PREGATHER[(z.device, z.data_ptr())] = (zb_all, keep)


def take_pregather(z: torch.Tensor):
    return _PREGATHER.pop((z.device, z.data_ptr()), None)


class _NTXentHipFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, n, temperature, reduction, gather, st):
        from ..ops import _ext
        ops = _ext.ops()
        R, D = z.shape
        dev = z.device
        zb = z.contiguous() if z.dtype == torch.bfloat16 else z.to(torch.bfloat16).contiguous()
        inv_t = 1.0 / temperature
        lse = torch.empty((R,), device=dev, dtype=torch.float32)
        rows = torch.empty((R,), device=dev, dtype=torch.float32)
        if gather and st.comm:
            # global negatives: the ranks exchange bf16 z (half the bytes of gathering fp32 ẑ) on
            # a side stream.  Meanwhile this rank normalises its own rows and scores them against
            # its OWN columns (their online log-sum-exp partials, the positive included); after
            # the exchange every rank normalises the peers' rows with the same row-wise kernel
            # (its copy of a peer's ẑ is bitwise the peer's own) and scores the remaining
            # columns into further split partials; one merge gives lse and the loss.
            W = st.world_size
            col_offset = st.rank * R
            Ccols = W * R
            cur = torch.cuda.current_stream(dev)
            side = _side_stream(dev)
            side.wait_stream(cur)
            pre = take_pregather(zb)
            if pre is not None and tuple(pre[0].shape) == (Ccols, D):
                # the head gathered z view by view on this side stream, under its GEMM 2
                zb_all, pre_keep = pre
            else:
                pre_keep = pre  # (a mismatched pre-gather's buffers: still in use on the side stream)
                zb_all = torch.empty((Ccols, D), device=dev, dtype=torch.bfloat16)
                with torch.cuda.stream(side):
                    ipc = getattr(st, "ipc", None)
                    if ipc is not None:  # one-shot stores over xGMI (comm/ipc.py, csrc/comm.hip)
                        ipc.all_gather(("ntxent", "z"), zb, zb_all)
                    else:
                        dist.all_gather_into_tensor(zb_all, zb, group=st.group)
            zall = torch.empty((Ccols, D), device=dev, dtype=torch.float32)
            inv_all = torch.empty((Ccols,), device=dev, dtype=torch.float32)
            zn = zall[col_offset:col_offset + R]
            inv = inv_all[col_offset:col_offset + R]
            znT = torch.empty((D, Ccols), device=dev, dtype=torch.float32)
            ops.nt_normalize(zb, zn, inv)
            ops.nt_transpose_cols(zn, znT, col_offset)
            s_loc = ops.nt_fwd_splits(R, R)
            s_rem = ops.nt_fwd_splits(R, Ccols - R)
            part = torch.empty(((s_loc + 2 * s_rem) * R * 3,), device=dev, dtype=torch.float32)
            ops.nt_forward_range(znT, R, col_offset, n, inv_t, part, col_offset, col_offset + R,
                                 s_loc, 0)  # overlaps the exchange
            cur.wait_stream(side)
            zb_all.record_stream(cur)
            del pre_keep  # (the head's per-view gather buffers: the side stream is joined)
            # every row in one launch each (this rank's block is rewritten with identical
            # values, after the local scoring read it: same stream)
            ops.nt_normalize(zb_all, zall, inv_all)
            ops.nt_transpose(zall, znT)
            nsp = s_loc
            for lo, hi in ((0, col_offset), (col_offset + R, Ccols)):
                if hi > lo:
                    sp = max(1, (s_rem * (hi - lo) + (Ccols - R) - 1) // (Ccols - R))
                    ops.nt_forward_range(znT, R, col_offset, n, inv_t, part, lo, hi, sp, nsp)
                    nsp += sp
            ops.nt_finish(part, R, nsp, lse, rows)
        else:
            zn = torch.empty((R, D), device=dev, dtype=torch.float32)
            inv = torch.empty((R,), device=dev, dtype=torch.float32)
            ops.nt_normalize(zb, zn, inv)
            zall = zn
            col_offset = 0
            Ccols = R
            znT = torch.empty((D, Ccols), device=dev, dtype=torch.float32)
            ops.nt_transpose(zall, znT)
            splits = ops.nt_fwd_splits(R, Ccols)
            part = torch.empty((splits * R * 3,), device=dev, dtype=torch.float32)
            ops.nt_forward(znT, R, col_offset, n, inv_t, part, splits, lse, rows)
        out = torch.empty((1,), device=dev, dtype=torch.float32)
        scale = 1.0 / R if reduction == "mean" else 1.0
        ops.nt_reduce_loss(rows, scale, out)
        ctx.save_for_backward(zn, zall, znT, lse, inv)
        ctx.cfg = (n, inv_t, scale, col_offset, gather, st, z.dtype)
        return out.view(())

    @staticmethod
    def backward(ctx, gout):
        from ..ops import _ext
        ops = _ext.ops()
        zn, zall, znT, lse, inv = ctx.saved_tensors
        n, inv_t, scale, col_offset, gather, st, zdtype = ctx.cfg
        R, D = zn.shape
        Ccols = zall.shape[0]
        dev = zn.device
        g = gout.reshape(1).float().contiguous()
        s_col = ops.nt_bwd_splits(Ccols, R)
        part2 = torch.empty((s_col * Ccols * D,), device=dev, dtype=torch.float32)
        d_cols = torch.empty((Ccols, D), device=dev, dtype=torch.float32)
        ops.nt_backward_part(False, zall, znT, lse, R, col_offset, n, inv_t, scale, g, part2,
                             s_col, d_cols)
        overlap = gather and st.comm and dev.type == "cuda"
        if overlap:
            # global negatives: only this rank's slice of the column gradient is needed, so a
            # reduce-scatter (1/W of an all-reduce's bytes over xGMI) — issued on a side stream
            # so it runs under the row-gradient kernel below
            cur = torch.cuda.current_stream(dev)
            side = _side_stream(dev)
            side.wait_stream(cur)
            mine = torch.empty((R, D), device=dev, dtype=torch.float32)
            with torch.cuda.stream(side):
                ipc = getattr(st, "ipc", None)
                if ipc is not None:
                    ipc.reduce_scatter(("ntxent", "dcols"), d_cols, mine)
                else:
                    dist.reduce_scatter_tensor(mine, d_cols, group=st.group)
            # (d_cols / mine stay referenced until the join below, which orders every later
            # allocation on this stream after the side stream's use)
        s_row = ops.nt_bwd_splits(R, Ccols)
        part = torch.empty((s_row * R * D,), device=dev, dtype=torch.float32)
        d_rows = torch.empty((R, D), device=dev, dtype=torch.float32)
        ops.nt_backward_part(True, zall, znT, lse, R, col_offset, n, inv_t, scale, g, part, s_row,
                             d_rows)
        if overlap:
            cur.wait_stream(side)
            d_rows += mine
        elif gather and st.comm:
            mine = torch.empty((R, D), device=dev, dtype=torch.float32)
            dist.reduce_scatter_tensor(mine, d_cols, group=st.group)
            d_rows += mine
        else:
            d_rows += d_cols[col_offset:col_offset + R]
        if zdtype == torch.bfloat16:
            dz = torch.empty((R, D), device=dev, dtype=torch.bfloat16)
            ops.nt_normalize_backward(zn, inv, d_rows, dz, None)
        else:
            dz = torch.empty((R, D), device=dev, dtype=torch.float32)
            ops.nt_normalize_backward(zn, inv, d_rows, None, dz)
        return dz, None, None, None, None, None


class NTXent(nn.Module):
    def __init__(self, temperature: float = 0.1, reduction: str = "mean",
                 device: Optional[torch.device] = None, gather=False):
        """``gather``: False (reference, per-GPU negatives), True (all-gathered global
        negatives, fused kernel) or ``"ring"`` (global negatives circulated around the ranks,
        loss/ring.py)."""
        assert temperature > 0.0
        assert reduction in {"none", "mean", "sum"}
        super().__init__()
        self.temperature = temperature
        self.reduction = reduction
        self.gather = "ring" if str(gather).lower() == "ring" else bool(gather)

    def forward(self, view0: torch.Tensor, view1: Optional[torch.Tensor] = None) -> torch.Tensor:
        """``forward(view0, view1)`` as the reference, or ``forward(z)`` with z = [view0; view1]."""
        if view1 is not None:
            z = torch.cat([view0, view1], dim=0)
            n = view0.shape[0]
        else:
            z = view0
            n = z.shape[0] // 2
        st = pstate.get()
        R, D = z.shape
        if self.gather == "ring" and st.comm and st.world_size > 1:
            # global negatives with the column blocks circulating around the ranks (loss/ring.py)
            from .ring import nt_xent_ring
            if self.reduction != "mean":
                raise ValueError("ring NT-Xent supports reduction='mean'")
            return nt_xent_ring(z, n, self.temperature, st.group, st.world_size, st.rank)
        if (z.is_cuda and self.reduction != "none" and registry.use_hip(z) and R % 16 == 0
                and D in (32, 64, 128, 256)):
            return _NTXentHipFn.apply(z, n, self.temperature, self.reduction, self.gather, st)
        return nt_xent_torch(z, n, self.temperature, self.reduction, self.gather, st.group,
                             st.world_size, st.rank)


# reference class name
NT_Xent = NTXent
