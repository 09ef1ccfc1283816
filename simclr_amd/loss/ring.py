"""Ring NT-Xent: global negatives without materialising the gathered embedding set.

``loss.gather=true`` all-gathers every rank's normalised embeddings (W·R×D) and scores each
local anchor against all of them in one fused kernel — ideal while W·R×D fits comfortably (8 GPUs
× 1024 rows × 128 = 4 MiB).  ``loss.gather=ring`` is the "ring attention" analogue for global
batches whose similarity blocks should never coexist: the column blocks travel around the ring of
ranks (point-to-point over xGMI, ``dist.batch_isend_irecv``) while each rank folds block t into an
online log-sum-exp of its anchors (running max / scaled sum, as flash attention does over key
blocks), receiving block t+1 during block t's matmul.  Memory per rank: two R×D blocks and one
R×R logit tile, independent of W.

Backward re-circulates the blocks with a gradient accumulator riding along: at every hop a rank
adds its anchors' contribution Σ_i p_ij·z_i to the accumulator of the block it holds and its own
row gradient Σ_j p_ij·z_j; after W hops each block is back home carrying the sum of every rank's
column gradient for it — the reduce-scatter of the gathered implementation, done in the ring.

Semantics are exactly those of the gathered loss (tests/test_distributed.py checks loss and
gradients against ``nt_xent_torch(gather=True)`` and a single process on the full batch): anchor i
of rank r sees every other row of the global batch, its positive is the other view of the same
image (a local row), the reduction is the mean over the rank's anchors.  Reference loss:
/root/reference/loss.py:25-65 (local only; the ring is an extension of the north star).
"""
from __future__ import annotations

from typing import List, Tuple

import torch
import torch.distributed as dist
import torch.nn.functional as F


def _peers(group, world: int, rank: int) -> Tuple[int, int]:
    nxt, prv = (rank + 1) % world, (rank - 1) % world
    if group is not None and group is not dist.group.WORLD:
        return dist.get_global_rank(group, nxt), dist.get_global_rank(group, prv)
    return nxt, prv


def _shift(tensors: List[torch.Tensor], group, world: int, rank: int):
    """Send ``tensors`` to the next rank and receive the previous rank's into new buffers;
    returns (buffers, requests)."""
    nxt, prv = _peers(group, world, rank)
    bufs = [torch.empty_like(t) for t in tensors]
    ops = []
    for t, b in zip(tensors, bufs):
        ops.append(dist.P2POp(dist.isend, t.contiguous(), nxt, group))
        ops.append(dist.P2POp(dist.irecv, b, prv, group))
    return bufs, dist.batch_isend_irecv(ops)


def _block_logits(zn: torch.Tensor, blk: torch.Tensor, inv_t: float, own: bool) -> torch.Tensor:
    L = (zn @ blk.t()) * inv_t
    if own:  # self similarity is not a candidate
        L.fill_diagonal_(float("-inf"))
    return L


class _RingNTXentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, n, temperature, group, world, rank):
        zf = z.float()
        norm = zf.norm(dim=1, keepdim=True).clamp_min(1e-12)
        zn = zf / norm
        R = zn.shape[0]
        inv_t = 1.0 / temperature
        idx = torch.arange(R, device=z.device)
        pos_col = torch.where(idx < n, idx + n, idx - n)
        m = torch.full((R,), float("-inf"), device=z.device)
        s = torch.zeros((R,), device=z.device)
        pos = None
        blk = zn
        for t in range(world):
            reqs = None
            if t < world - 1:
                (nxt_blk,), reqs = _shift([blk], group, world, rank)
            L = _block_logits(zn, blk, inv_t, own=(t == 0))
            if t == 0:
                pos = L[idx, pos_col]
            m_new = torch.maximum(m, L.max(dim=1).values)
            s = s * torch.exp(m - m_new) + torch.exp(L - m_new[:, None]).sum(dim=1)
            m = m_new
            if reqs is not None:
                for r in reqs:
                    r.wait()
                blk = nxt_blk
        lse = m + torch.log(s)
        loss = (lse - pos).mean()
        ctx.save_for_backward(zn, norm, lse)
        ctx.cfg = (n, inv_t, group, world, rank, z.dtype)
        return loss

    @staticmethod
    def backward(ctx, gout):
        zn, norm, lse = ctx.saved_tensors
        n, inv_t, group, world, rank, zdtype = ctx.cfg
        R = zn.shape[0]
        idx = torch.arange(R, device=zn.device)
        pos_col = torch.where(idx < n, idx + n, idx - n)
        g = gout.float() * inv_t / R
        d_rows = torch.zeros_like(zn)
        blk, acc = zn, torch.zeros_like(zn)
        for t in range(world):
            P = torch.exp(_block_logits(zn, blk, inv_t, own=(t == 0)) - lse[:, None])
            if t == 0:
                P[idx, pos_col] -= 1.0  # the positive's −1 of the softmax cross-entropy
            d_rows += g * (P @ blk)
            acc = acc + g * (P.t() @ zn)
            if world > 1:
                (blk, acc), reqs = _shift([blk, acc], group, world, rank)
                for r in reqs:
                    r.wait()
        dzn = d_rows + acc  # after W hops ``acc`` is this rank's own block's column gradient
        dz = (dzn - zn * (zn * dzn).sum(dim=1, keepdim=True)) / norm
        return dz.to(zdtype), None, None, None, None, None


def nt_xent_ring(z: torch.Tensor, n: int, temperature: float, group=None, world: int = 1,
                 rank: int = 0) -> torch.Tensor:
    """Mean NT-Xent of this rank's anchors against the whole global batch, ring-circulated."""
    if world <= 1:
        from .ntxent import nt_xent_torch
        return nt_xent_torch(z, n, temperature, "mean")
    return _RingNTXentFn.apply(z, n, temperature, group, world, rank)
