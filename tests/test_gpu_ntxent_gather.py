"""The gathered-negatives HIP NT-Xent path (``loss.gather=true``; north star) in ONE
process: the rank's rows are scored against W·R columns of which W−1 blocks are synthesised
"peer" embeddings, with ``col_offset = r·R`` ≠ 0.  The collectives of loss/ntxent.py are
replaced by in-process fakes (all-gather = concatenation with the peer blocks, reduce-scatter =
this rank's slice of the column gradient, as if every peer contributed zero), so the loss, the
row gradient and the full column gradient of the kernels (nt_forward / nt_backward_part with
Ccols = W·R) are compared with an fp32 torch oracle of the same global-column loss
(/root/reference/loss.py:33-65 with the columns extended)."""
import types

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _oracle(z_local, peers, r, n, tau):
    """fp32 NT-Xent of the local rows against [peer blocks with the local block at r]."""
    R = z_local.shape[0]
    blocks = [p for p in peers]
    blocks.insert(r, z_local)
    zall = torch.cat(blocks)
    zn_all = F.normalize(zall.float(), dim=1)
    zn = zn_all[r * R:(r + 1) * R]
    sim = zn @ zn_all.t() / tau
    idx = torch.arange(R, device=zall.device)
    sim[idx, r * R + idx] = float("-inf")
    tgt = r * R + torch.where(idx < n, idx + n, idx - n)
    return F.cross_entropy(sim, tgt, reduction="sum") / n * 0.5


@pytest.mark.parametrize("W,r", [(2, 0), (2, 1), (8, 0), (8, 7), (8, 3)])
def test_gathered_ntxent_kernel_path(monkeypatch, W, r):
    from simclr_amd.loss import ntxent as mod
    from simclr_amd.ops import _ext
    _ext.require()
    n, D, tau = 256, 128, 0.5
    R = 2 * n
    g = torch.Generator(device=DEV).manual_seed(100 * W + r)
    z = torch.randn(R, D, device=DEV, generator=g).to(torch.bfloat16)
    # peers: correlated with this rank's rows so some peer columns are hard negatives
    peers = [(0.6 * z.float() + 0.8 * torch.randn(R, D, device=DEV, generator=g))
             .to(torch.bfloat16) for _ in range(W - 1)]
    seen = {}

    def fake_all_gather(out, inp, group=None):
        blocks = list(peers)
        blocks.insert(r, inp)
        out.copy_(torch.cat(blocks))

    def fake_reduce_scatter(out, inp, group=None):
        seen["d_cols"] = inp.clone()
        out.copy_(inp[r * R:(r + 1) * R])

    monkeypatch.setattr(mod.dist, "all_gather_into_tensor", fake_all_gather)
    monkeypatch.setattr(mod.dist, "reduce_scatter_tensor", fake_reduce_scatter)
    st = types.SimpleNamespace(comm=True, world_size=W, rank=r, group=None)
    monkeypatch.setattr(mod.pstate, "get", lambda: st)

    zh = z.clone().requires_grad_(True)
    loss = mod.NTXent(tau, gather=True)(zh)
    loss.backward()
    torch.cuda.synchronize()

    zr = z.float().requires_grad_(True)
    pr = [p.float().requires_grad_(True) for p in peers]
    lr = _oracle(zr, pr, r, n, tau)
    lr.backward()
    assert abs(float(loss) - float(lr)) < 2e-4 * max(1.0, abs(float(lr))), (float(loss), float(lr))

    def rel(a, b):
        return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))
    # the rank's own gradient (row terms + its column block); bf16 output rounding only
    assert rel(zh.grad, zr.grad) < 1e-2, rel(zh.grad, zr.grad)
    # the column gradient the kernels send to the peers, in normalised space: compare through
    # the normalisation Jacobian of each peer block
    dc = seen["d_cols"]
    for j, (p, pg) in enumerate(zip(peers, pr)):
        blk = j if j < r else j + 1
        pn = F.normalize(p.float(), dim=1)
        inv = 1.0 / p.float().norm(dim=1, keepdim=True)
        d = dc[blk * R:(blk + 1) * R]
        dz = (d - pn * (pn * d).sum(1, keepdim=True)) * inv
        assert rel(dz, pg.grad) < 1e-3, (blk, rel(dz, pg.grad))
