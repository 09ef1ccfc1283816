"""Fused 1x1 backward (csrc/conv.hip conv1x1_bwd_dual): a bottleneck conv3's dgrad (with the BN2
ReLU-mask epilogue and the BN2-backward Σg / Σg·x̂ partials) and its weight gradient from ONE
pass over the output gradient, with and without the lazy BN3-backward prologue
(dY = A·g + B·a3 + D per view segment), against an fp32 PyTorch reference of the same math
(/root/reference/model.py Bottleneck.conv3 under SyncBatchNorm)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _bf(t):
    return t.to(torch.bfloat16)


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


@pytest.mark.parametrize("dual8", [False, True])
@pytest.mark.parametrize("Nb,H,lazy,bps", [(64, 8, True, 32), (64, 8, False, 16),
                                           (32, 32, True, 128), (32, 32, False, 64)])
def test_conv1x1_bwd_dual_matches_fp32(Nb, H, lazy, bps, dual8):
    """(dual8: the same op as the 8-wave, 64-row-tile conv1x1_bwd_dual_w form.)"""
    from simclr_amd.ops import _ext
    ops = _ext.ops()
    torch.manual_seed(Nb + H + int(lazy))
    S, Co, Ci = 2, 256, 64
    M = Nb * H * H
    seg = M // S
    G = _bf(torch.randn(M, Co, device=DEV))
    A3 = _bf(torch.randn(M, Co, device=DEV)) if lazy else None
    coef = torch.randn(3, S, Co, device=DEV) * 0.5 if lazy else None
    X = _bf(torch.randn(M, Ci, device=DEV))
    ss = torch.stack([0.5 + torch.rand(S, Ci, device=DEV), torch.randn(S, Ci, device=DEV) * 0.3])
    mi = torch.stack([torch.randn(S, Ci, device=DEV) * 0.1, 0.5 + torch.rand(S, Ci, device=DEV)])
    W = _bf(torch.randn(Co, Ci, device=DEV) * 0.06)        # conv3 weight [Co][Ci] (1x1)
    Wt = W.t().contiguous()                                 # dgrad operand [Ci][Co]
    gm = torch.empty(M, Ci, device=DEV, dtype=torch.bfloat16)
    stats = torch.empty(S * bps * 2 * Ci, device=DEV)
    wpart = torch.empty(S * bps * Co * Ci, device=DEV)
    ops.conv1x1_bwd_dual(G, A3, coef.reshape(-1) if lazy else None, X, ss.reshape(-1),
                         mi.reshape(-1), Wt, gm, stats, wpart, S, bps, dual8=dual8)
    dW = torch.empty(Co, Ci, device=DEV)
    ops.wgrad_reduce_slabs(wpart, S * bps, dW)
    torch.cuda.synchronize()

    # fp32 reference (operands rounded to bf16 where the kernel rounds them)
    sg = torch.arange(M, device=DEV) // seg
    if lazy:
        dY = _bf(coef[0][sg] * G.float() + coef[1][sg] * A3.float() + coef[2][sg]).float()
    else:
        dY = G.float()
    Xf = X.float()
    Xp = _bf(torch.relu(Xf * ss[0][sg] + ss[1][sg])).float()
    dX = _bf(dY @ W.float()).float()
    mask = (Xf * ss[0][sg] + ss[1][sg]) > 0
    g = torch.where(mask, dX, torch.zeros_like(dX))
    xh = (Xf - mi[0][sg]) * mi[1][sg]
    st = stats.view(S, bps, 2, Ci).sum(1)
    ref_s1 = torch.stack([g[sg == s].sum(0) for s in range(S)])
    ref_s2 = torch.stack([(g * xh)[sg == s].sum(0) for s in range(S)])
    dW_ref = dY.t() @ Xp
    assert _rel(gm, g) < 1e-2, _rel(gm, g)
    # masks agree exactly: every zero of the reference is a zero of the kernel
    assert int(((gm.float() != 0) & ~mask).sum()) == 0
    assert _rel(st[:, 0], ref_s1) < 2e-3, _rel(st[:, 0], ref_s1)
    assert _rel(st[:, 1], ref_s2) < 2e-3, _rel(st[:, 1], ref_s2)
    assert _rel(dW, dW_ref) < 2e-3, _rel(dW, dW_ref)


@pytest.mark.parametrize("Nb,H,lazy,pre,bps", [(64, 16, True, True, 64), (64, 16, True, False, 64),
                                               (32, 16, False, True, 32), (16, 8, False, False, 8),
                                               (1024, 16, True, True, 64)])
def test_conv1x1_bwd_dual_wide_matches_fp32(Nb, H, lazy, pre, bps):
    """The wide form (Co = 512, Ci = 128: ResNet-50 layer2 conv3; two 64-channel Ci slices per
    row block, 32-row tiles, 8 waves) with and without the lazy BN3 prologue, with X either
    BN2-applied in the kernel or the forward's materialised relu(bn2(a2)) (``Xraw`` = a2 for the
    epilogue), against fp32 torch: dX with the BN2 mask, the BN2-backward partials, dW.
    (1024, 16): the production layer2 shape (512 images x 2 views)."""
    from simclr_amd.ops import _ext
    ops = _ext.ops()
    torch.manual_seed(Nb + H + int(lazy) + 2 * int(pre))
    S, Co, Ci = 2, 512, 128
    M = Nb * H * H
    seg = M // S
    G = _bf(torch.randn(M, Co, device=DEV))
    A3 = _bf(torch.randn(M, Co, device=DEV)) if lazy else None
    coef = torch.randn(3, S, Co, device=DEV) * 0.5 if lazy else None
    X = _bf(torch.randn(M, Ci, device=DEV))              # a2 (pre-BN)
    ss = torch.stack([0.5 + torch.rand(S, Ci, device=DEV), torch.randn(S, Ci, device=DEV) * 0.3])
    mi = torch.stack([torch.randn(S, Ci, device=DEV) * 0.1, 0.5 + torch.rand(S, Ci, device=DEV)])
    W = _bf(torch.randn(Co, Ci, device=DEV) * 0.04)
    Wt = W.t().contiguous()
    sg = torch.arange(M, device=DEV) // seg
    Xf = X.float()
    Xp = _bf(torch.relu(Xf * ss[0][sg] + ss[1][sg]))    # what the forward materialises
    gm = torch.full((M, Ci), float("nan"), device=DEV, dtype=torch.bfloat16)
    stats = torch.full((S * bps * 2 * Ci,), float("nan"), device=DEV)
    wpart = torch.full((S * bps * Co * Ci,), float("nan"), device=DEV)
    ops.conv1x1_bwd_dual(G, A3, coef.reshape(-1) if lazy else None, Xp if pre else X,
                         ss.reshape(-1), mi.reshape(-1), Wt, gm, stats, wpart, S, bps,
                         X if pre else None)
    dW = torch.empty(Co, Ci, device=DEV)
    ops.wgrad_reduce_slabs(wpart, S * bps, dW)
    torch.cuda.synchronize()
    if lazy:
        dY = _bf(coef[0][sg] * G.float() + coef[1][sg] * A3.float() + coef[2][sg]).float()
    else:
        dY = G.float()
    dX = _bf(dY @ W.float()).float()
    mask = (Xf * ss[0][sg] + ss[1][sg]) > 0
    g = torch.where(mask, dX, torch.zeros_like(dX))
    xh = (Xf - mi[0][sg]) * mi[1][sg]
    st = stats.view(S, bps, 2, Ci).sum(1)
    ref_s1 = torch.stack([g[sg == s].sum(0) for s in range(S)])
    ref_s2 = torch.stack([(g * xh)[sg == s].sum(0) for s in range(S)])
    dW_ref = dY.t() @ Xp.float()
    assert _rel(gm, g) < 1e-2, _rel(gm, g)
    assert int(((gm.float() != 0) & ~mask).sum()) == 0
    assert _rel(st[:, 0], ref_s1) < 2e-3, _rel(st[:, 0], ref_s1)
    assert _rel(st[:, 1], ref_s2) < 2e-3, _rel(st[:, 1], ref_s2)
    assert _rel(dW, dW_ref) < 2e-3, _rel(dW, dW_ref)


@pytest.mark.parametrize("dual8", [False, True])
@pytest.mark.parametrize("Nb,H,lazy,bps", [(64, 8, True, 32), (32, 32, True, 128),
                                           (32, 16, False, 64)])
def test_conv1x1_bwd_dual_plain_matches_fp32(Nb, H, lazy, bps, dual8):
    """The plain form (a stride-1 1x1 downsample, layer1.0: no BatchNorm between its input and
    the conv, so no X transform, no mask, no partials): dX = dY · W unmasked and dW = dYᵀ · X,
    with dY the downsample BN's backward A·g + B·ad + D formed in registers, vs fp32 torch."""
    from simclr_amd.ops import _ext
    ops = _ext.ops()
    torch.manual_seed(Nb * H + int(lazy))
    S, Co, Ci = 2, 256, 64
    M = Nb * H * H
    seg = M // S
    G = _bf(torch.randn(M, Co, device=DEV))
    A3 = _bf(torch.randn(M, Co, device=DEV)) if lazy else None
    coef = torch.randn(3, S, Co, device=DEV) * 0.5 if lazy else None
    X = _bf(torch.relu(torch.randn(M, Ci, device=DEV)))  # a block input (post-ReLU)
    W = _bf(torch.randn(Co, Ci, device=DEV) * 0.06)
    Wt = W.t().contiguous()
    gm = torch.full((M, Ci), float("nan"), device=DEV, dtype=torch.bfloat16)
    wpart = torch.full((S * bps * Co * Ci,), float("nan"), device=DEV)
    ops.conv1x1_bwd_dual(G, A3, coef.reshape(-1) if lazy else None, X, None, None, Wt, gm,
                         torch.empty(1, device=DEV), wpart, S, bps, dual8=dual8)
    dW = torch.empty(Co, Ci, device=DEV)
    ops.wgrad_reduce_slabs(wpart, S * bps, dW)
    torch.cuda.synchronize()
    sg = torch.arange(M, device=DEV) // seg
    if lazy:
        dY = _bf(coef[0][sg] * G.float() + coef[1][sg] * A3.float() + coef[2][sg]).float()
    else:
        dY = G.float()
    assert _rel(gm, dY @ W.float()) < 1e-2, _rel(gm, dY @ W.float())
    assert _rel(dW, dY.t() @ X.float()) < 2e-3, _rel(dW, dY.t() @ X.float())


@pytest.mark.parametrize("Nb,H,bps", [(16, 8, 2), (64, 32, 32), (1024, 32, 32)])
def test_conv1x1_bwd_dual_s2_matches_fp32(Nb, H, bps):
    """The strided plain wide form (layer2.0's 1x1 stride-2 downsample, Co 512 / Ci 256): the
    compact input gradient (the even input positions only) and the weight gradient from one
    pass over dY, X read at the even positions of the block input, vs fp32 torch conv2d
    gradients.  (1024, 32): the production shape."""
    import torch.nn.functional as F
    from simclr_amd.ops import _ext
    ops = _ext.ops()
    torch.manual_seed(Nb + H)
    S, Co, Ci = 2, 512, 256
    OH = (H + 1) // 2
    Mo = Nb * OH * OH
    X = _bf(torch.relu(torch.randn(Nb, H, H, Ci, device=DEV)))
    dY = _bf(torch.randn(Nb, OH, OH, Co, device=DEV))
    W = _bf(torch.randn(Co, Ci, device=DEV) * 0.04)
    Wt = W.t().contiguous()
    gm = torch.full((Nb, OH, OH, Ci), float("nan"), device=DEV, dtype=torch.bfloat16)
    wpart = torch.full((S * bps * Co * Ci,), float("nan"), device=DEV)
    ops.conv1x1_bwd_dual_s2(dY, None, None, X, Wt, gm, wpart, S, bps)
    dW = torch.empty(Co, Ci, device=DEV)
    ops.wgrad_reduce_slabs(wpart, S * bps, dW)
    torch.cuda.synchronize()
    xr = X.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = W.float().view(Co, Ci, 1, 1).requires_grad_(True)
    F.conv2d(xr, wr, None, 2, 0).backward(dY.float().permute(0, 3, 1, 2))
    ref_dx = xr.grad.permute(0, 2, 3, 1)[:, ::2, ::2, :]
    assert _rel(gm, ref_dx) < 1e-2, _rel(gm, ref_dx)
    assert _rel(dW, wr.grad.view(Co, Ci)) < 2e-3, _rel(dW, wr.grad.view(Co, Ci))
