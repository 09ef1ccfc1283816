"""Fused ResNet-stage executor (``simclr_amd/models/fused.py``) and the kernel features it uses:
the mode-3 dgrad epilogue (ReLU mask + BatchNorm-backward partials, segment-major stats remap
across the stride-2 parity classes), ``bn_apply_ss`` and the finalize scale/shift table — each
against a plain PyTorch fp32 reference — and the whole executor against the per-module path."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module")
def ops():
    from simclr_amd.ops import _ext
    _ext.require()
    return torch.ops.simclr_amd


def _bf(t):
    return t.to(torch.bfloat16)


def _rel(a, b):
    return (a.float() - b.float()).abs().max().item() / (b.float().abs().max().item() + 1e-6)


@pytest.mark.parametrize("k,s,p", [(1, 1, 0), (3, 1, 1), (3, 2, 1)])
def test_dgrad_mode3_epilogue(ops, k, s, p):
    from simclr_amd.models.fused import FusedStages, _BNState, _ConvSpec
    torch.manual_seed(3)
    N, Ci, H, W, Co, S = 8, 64, 16, 16, 128, 2
    conv = torch.nn.Conv2d(Ci, Co, k, s, p, bias=False).to(DEV)
    with torch.no_grad():
        conv.weight.copy_(_bf(torch.randn_like(conv.weight) / math.sqrt(Ci * k * k)).float())
    OH = (H + 2 * p - k) // s + 1
    dy = _bf(torch.randn(N, OH, OH, Co, device=DEV))
    a_prev = _bf(torch.randn(N, H, W, Ci, device=DEV))
    sc = torch.rand(S, Ci, device=DEV) + 0.5
    sh = torch.randn(S, Ci, device=DEV) * 0.3
    mean = torch.randn(S, Ci, device=DEV) * 0.2
    inv = torch.rand(S, Ci, device=DEV) + 0.5
    bs = _BNState(torch.cat([mean, inv]).reshape(-1).contiguous(),
                  torch.stack([sc, sh]).reshape(2, S * Ci).contiguous(), 1.0)
    ex = FusedStages.__new__(FusedStages)
    cs = _ConvSpec(conv, None, s, k, p)
    gm, part, nb = ex._dgrad(ops, dy, cs, a_prev.shape, S, bn_epi=("mask", a_prev, bs))
    sums = torch.empty(2 * S * Ci, device=DEV)
    ops.bn_reduce(part, nb, S, Ci, sums)
    # fp32 reference
    dx = torch.nn.grad.conv2d_input((N, Ci, H, W), conv.weight.float(),
                                    dy.permute(0, 3, 1, 2).float(), s, p)
    dx = _bf(dx).float().permute(0, 2, 3, 1)
    seg = (torch.arange(N, device=DEV) // (N // S))[:, None, None, None]
    af = a_prev.float()
    mask = af * sc[seg.squeeze()][:, None, None, :] + sh[seg.squeeze()][:, None, None, :] > 0
    g = torch.where(mask, dx, 0.0)
    assert _rel(gm, g) < 2e-2
    xh = (af - mean[seg.squeeze()][:, None, None, :]) * inv[seg.squeeze()][:, None, None, :]
    gk = gm.float()  # the kernel's (bf16) g drives its own sums: compare against them
    ref1 = gk.reshape(S, -1, Ci).sum(1)
    ref2 = (gk * xh).reshape(S, -1, Ci).sum(1)
    got = sums.view(2, S, Ci)
    assert _rel(got[0], ref1) < 1e-3
    assert _rel(got[1], ref2) < 1e-3


@pytest.mark.parametrize("N,H,Ci,Co", [(8, 16, 64, 256), (32, 4, 512, 2048)])
def test_bn_backward_operand_prologue(ops, N, H, Ci, Co):
    """conv3's dgrad (PRO=2) and wgrad (DPRO) computing da = A·g + B·a + D in the operand
    prologue == materialising da with ``bn_bwd_apply`` first (and both vs fp32)."""
    from simclr_amd.models.fused import FusedStages, _BNState, _ConvSpec
    torch.manual_seed(4)
    S = 2
    conv = torch.nn.Conv2d(Ci, Co, 1, 1, 0, bias=False).to(DEV)
    with torch.no_grad():
        conv.weight.copy_(_bf(torch.randn_like(conv.weight) / math.sqrt(Ci)).float())
    g = _bf(torch.randn(N, H, H, Co, device=DEV))
    a = _bf(torch.randn(N, H, H, Co, device=DEV))
    xin = _bf(torch.randn(N, H, H, Ci, device=DEV))
    coef = torch.randn(3 * S * Co, device=DEV) * 0.5
    a_prev = _bf(torch.randn(N, H, H, Ci, device=DEV))
    sc = torch.rand(S, Ci, device=DEV) + 0.5
    sh = torch.randn(S, Ci, device=DEV) * 0.3
    mi = torch.cat([torch.randn(S, Ci, device=DEV) * 0.2, torch.rand(S, Ci, device=DEV) + 0.5])
    bs = _BNState(mi.reshape(-1).contiguous(), torch.stack([sc, sh]).reshape(2, S * Ci).contiguous(), 1.0)
    ex = FusedStages.__new__(FusedStages)
    ex.bnb_prologue = True
    cs = _ConvSpec(conv, None, 1, 1, 0)
    assert ex._bnb_ok(cs, a, S) == (Ci <= 128)  # the kernels below run regardless
    da = torch.empty_like(a)
    ops.bn_bwd_apply(g, None, a, coef, S, False, da, None)
    c = coef.view(3, S, 1, Co)
    ref_da = (c[0] * g.float().view(S, -1, Co) + c[1] * a.float().view(S, -1, Co) + c[2])
    assert _rel(da, ref_da.view_as(da)) < 1e-2
    gm0, p0, nb0 = ex._dgrad(ops, da, cs, a_prev.shape, S, bn_epi=("mask", a_prev, bs))
    gm1, p1, nb1 = ex._dgrad(ops, g, cs, a_prev.shape, S, bn_epi=("mask", a_prev, bs),
                             bnb=(a, coef))
    assert _rel(gm1, gm0) < 1e-2
    s0 = torch.empty(2 * S * Ci, device=DEV)
    s1 = torch.empty(2 * S * Ci, device=DEV)
    ops.bn_reduce(p0, nb0, S, Ci, s0)
    ops.bn_reduce(p1, nb1, S, Ci, s1)
    assert _rel(s1, s0) < 2e-2
    for bnb, dyn in ((None, da), ((a, coef), g)):
        conv.weight.grad = None
        ex._wgrad(ops, dyn, xin, cs, bs.ss, S, bnb=bnb)
        if bnb is None:
            w0 = conv.weight.grad.clone()
        else:
            w1 = conv.weight.grad.clone()
    xa = torch.relu(xin.float().view(S, -1, Ci) * sc[:, None] + sh[:, None]).reshape(-1, Ci)
    wref = ref_da.reshape(-1, Co).t() @ _bf(xa).float()
    assert _rel(w0.view(Co, Ci), wref) < 2e-2
    assert _rel(w1.view(Co, Ci), w0.view(Co, Ci)) < 1e-2


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_bn_apply_ss_and_finalize_table(ops, mode):
    torch.manual_seed(1)
    S, R, C = 2, 4096, 256
    x = _bf(torch.randn(S * R, C, device=DEV))
    res = _bf(torch.randn(S * R, C, device=DEV))
    stats = torch.stack([x.float().view(S, R, C).sum(1), (x.float() ** 2).view(S, R, C).sum(1)])
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV)
    mi = torch.empty(2 * S * C, device=DEV)
    ss = torch.empty(2 * S * C, device=DEV)
    ops.bn_finalize(stats.reshape(-1).contiguous(), S, C, float(R), 1e-5, 0.1, None, None, mi,
                    None, gamma, beta, ss)
    mean = stats[0] / R
    var = stats[1] / R - mean ** 2
    scale = gamma * torch.rsqrt(var + 1e-5)
    shift = beta - mean * scale
    assert torch.allclose(ss.view(2, S, C)[0], scale, rtol=1e-4, atol=1e-5)
    assert torch.allclose(ss.view(2, S, C)[1], shift, rtol=1e-4, atol=1e-4)
    y = torch.empty_like(x)
    rss = torch.stack([torch.rand(S, C, device=DEV), torch.randn(S, C, device=DEV)]).contiguous()
    ref = x.float().view(S, R, C) * scale[:, None] + shift[:, None]
    if mode == 0:
        ops.bn_apply_ss(x, ss, None, None, y, S, True)
    elif mode == 1:
        ops.bn_apply_ss(x, ss, res, None, y, S, True)
        ref = ref + res.float().view(S, R, C)
    else:
        ops.bn_apply_ss(x, ss, res, rss.view(-1), y, S, True)
        ref = ref + res.float().view(S, R, C) * rss[0][:, None] + rss[1][:, None]
    ref = torch.relu(ref).reshape(S * R, C)
    assert _rel(y, ref) < 1e-2
    # optional ReLU bitmask: bit e of byte (r, c // 8) == (y[r, c] > 0)
    mask = torch.empty(S * R * C // 8, device=DEV, dtype=torch.uint8)
    y2 = torch.empty_like(x)
    if mode == 0:
        ops.bn_apply_ss(x, ss, None, None, y2, S, True, mask)
    elif mode == 1:
        ops.bn_apply_ss(x, ss, res, None, y2, S, True, mask)
    else:
        ops.bn_apply_ss(x, ss, res, rss.view(-1), y2, S, True, mask)
    assert torch.equal(y2, y)
    bits = (y.float() > 0).view(-1, 8).to(torch.int32)
    packed = (bits << torch.arange(8, device=DEV, dtype=torch.int32)).sum(1)
    assert torch.equal(mask.to(torch.int32), packed)


@pytest.mark.parametrize("base,stem,batch,block_out", [("resnet50", True, 32, False),
                                                       ("resnet18", None, 64, False),
                                                       ("resnet50", True, 64, False),
                                                       ("resnet50", True, 64, True)])
def test_fused_stages_match_fp32(base, stem, batch, block_out, monkeypatch):
    """The fused executor vs fp32 torch and vs the per-module bf16 path on a well-conditioned
    network (tests/_fused_compare.py: damped residual branches, ReLU inputs away from zero,
    a projection loss on the backbone features): stage outputs, stage input gradients, running
    statistics and parameter gradients within the calibrated bounds of _fused_compare.py."""
    from _fused_compare import run_three, summary, violations
    mt = run_three(base, stem, batch, monkeypatch, block_out=block_out)
    print("FUSED-CHECK", base, batch, block_out, summary(mt))
    nblk, dual, outs = mt["launch_counts"]
    if block_out:  # every 1x1 conv1 after the first block formed its input itself
        assert (dual, outs) == (nblk - 1, 1), (dual, outs)
    else:
        assert (dual, outs) == (0, nblk), (dual, outs)
    assert mt["bstage"] and len(mt["stage"]) == 4
    bad = violations(mt)
    assert not bad, bad[:8]


@pytest.mark.parametrize("mutate", [("fwd", "layer3.1", 1), ("fwd", "layer3.0", 2),
                                    ("dgrad", "layer3.1", 1), ("dgrad", "layer2.2", 0)])
def test_fused_check_catches_two_percent_defect(mutate, monkeypatch):
    """Sensitivity of the check above: one conv of the fused executor made 2 % wrong — its
    forward output after the BatchNorm statistics were taken (what its consumers read), or its
    input gradient — must break at least one bound (measured margins: _fused_compare.py)."""
    from _fused_compare import run_three, summary, violations
    mt = run_three("resnet50", True, 32, monkeypatch, mutate=mutate)
    bad = violations(mt)
    print("MUTATION", mutate, len(bad), bad[:4], summary(mt))
    assert bad, f"a 2 % defect ({mutate}) passed the fused-executor check"


@pytest.mark.parametrize("C,nblk,S", [(64, 1, 2), (256, 33, 2), (2048, 512, 2), (512, 200, 1)])
def test_bn_reduce_fused_matches_three_launch_path(ops, C, nblk, S):
    """Single-launch last-arriver reduction == reduce → finalize (fwd and bwd), repeated so the
    ticket reset between launches is exercised; running stats / num_batches_tracked too."""
    torch.manual_seed(C + nblk)
    count = float(nblk * 64)
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV)
    for rep in range(3):
        part = torch.randn(S * nblk * 2 * C, device=DEV)
        part.view(S, nblk, 2, C)[:, :, 1].abs_().mul_(4.0)  # Σx² dominates (positive var)
        stats = torch.empty(2 * S * C, device=DEV)
        ops.bn_reduce(part, nblk, S, C, stats)
        st2 = torch.empty(2 * S * C, device=DEV)
        ops.bn_reduce_fused(part, nblk, S, C, 0, st2)
        assert torch.allclose(st2, stats, rtol=1e-5, atol=1e-4)
        rm0, rv0 = torch.randn(C, device=DEV), torch.rand(C, device=DEV) + 0.5
        nb0 = torch.zeros((), dtype=torch.long, device=DEV)
        rm1, rv1, nb1 = rm0.clone(), rv0.clone(), nb0.clone()
        mi0, ss0 = torch.empty(2 * S * C, device=DEV), torch.empty(2 * S * C, device=DEV)
        mi1, ss1 = torch.empty_like(mi0), torch.empty_like(ss0)
        ops.bn_finalize(stats, S, C, count, 1e-5, 0.1, rm0, rv0, mi0, nb0, gamma, beta, ss0)
        ops.bn_reduce_fused(part, nblk, S, C, 1, None, count, 1e-5, 0.1, rm1, rv1, mi1, nb1,
                            gamma, beta, ss1)
        for u, v in ((mi1, mi0), (ss1, ss0), (rm1, rm0), (rv1, rv0)):
            assert torch.allclose(u, v, rtol=1e-4, atol=1e-4)
        assert int(nb1) == int(nb0) == S
        coef0, coef1 = torch.empty(3 * S * C, device=DEV), torch.empty(3 * S * C, device=DEV)
        dg0, db0 = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        dg1, db1 = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        ops.bn_bwd_finalize(stats, mi0, gamma, S, C, count, dg0, db0, coef0)
        # mode 0 with dγ, dβ (the distributed backward: local sums + parameter gradients in one
        # launch, the sums all-reduced afterwards)
        st3 = torch.empty(2 * S * C, device=DEV)
        dg2, db2 = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        ops.bn_reduce_fused(part, nblk, S, C, 0, st3, dgamma=dg2, dbeta=db2)
        assert torch.allclose(st3, stats, rtol=1e-5, atol=1e-4)
        assert torch.allclose(dg2, dg0, rtol=1e-4, atol=1e-3)
        assert torch.allclose(db2, db0, rtol=1e-4, atol=1e-3)
        ops.bn_reduce_fused(part, nblk, S, C, 2, None, count, 0.0, 0.0, None, None, mi0, None,
                            gamma, None, None, dg1, db1, coef1)
        for u, v in ((coef1, coef0), (dg1, dg0), (db1, db0)):
            assert torch.allclose(u, v, rtol=1e-4, atol=1e-3)


def test_weight_transform_batch_matches_single(ops):
    """One batched launch == the per-conv dgrad weight transforms (bitwise), for stride-1 flips
    and stride-2 parity sub-kernels of 1x1 / 3x3 convs."""
    from simclr_amd.models.fused import FusedStages, _ConvSpec
    torch.manual_seed(2)
    specs = [(64, 64, 3, 1, 1), (256, 64, 1, 1, 0), (128, 256, 3, 2, 1), (512, 256, 1, 2, 0),
             (2048, 512, 1, 1, 0), (8, 16, 3, 2, 1)]
    Ws, Wts, params, refs = [], [], [], []
    for Co, Ci, k, s, p in specs:
        conv = torch.nn.Conv2d(Ci, Co, k, s, p, bias=False)
        w = _bf(torch.randn(Co, k, k, Ci, device=DEV))
        for key, prm in FusedStages._wt_params(_ConvSpec(conv, None, s, k, p)):
            ref = torch.empty((prm[3], prm[4], prm[5], prm[0]), device=DEV, dtype=torch.bfloat16)
            ops.weight_transform(w, ref, prm)
            Ws.append(w)
            Wts.append(torch.full_like(ref, float("nan")))
            params.extend(prm)
            refs.append(ref)
    plan = ops.weight_transform_plan(Ws, Wts, params)
    ops.weight_transform_batch(plan[:-1].to(DEV), int(plan[-1]))
    for got, ref in zip(Wts, refs):
        assert torch.equal(got, ref)


@pytest.mark.parametrize("H,mode", [(16, 1), (7, 1), (16, 4)])
def test_compact_downsample_residual(ops, H, mode):
    """A stride-2 1x1 downsample's dgrad kept compact ([N, ceil(H/2), ceil(W/2), C], one
    stride-1 GEMM) and added by conv1's dgrad epilogue through the subsampled-residual mode
    (epi_mode | 256) == the zero-filled full-resolution residual, bitwise: the same bf16
    values are added at the even positions, nothing elsewhere."""
    from simclr_amd.models.fused import FusedStages, _BNState, _ConvSpec
    torch.manual_seed(11)
    N, Cin, Cmid, Cds, S = 8, 64, 64, 128, 2
    conv1 = torch.nn.Conv2d(Cin, Cmid, 1, 1, 0, bias=False).to(DEV)
    down = torch.nn.Conv2d(Cin, Cds, 1, 2, 0, bias=False).to(DEV)
    for c in (conv1, down):
        with torch.no_grad():
            c.weight.copy_(_bf(torch.randn_like(c.weight) * 0.1).float())
    OHd = (H + 1) // 2
    da = _bf(torch.randn(N, H, H, Cmid, device=DEV))       # conv1 output gradient
    dad = _bf(torch.randn(N, OHd, OHd, Cds, device=DEV))   # downsample output gradient
    ex = FusedStages.__new__(FusedStages)
    cs1, csd = _ConvSpec(conv1, None, 1, 1, 0), _ConvSpec(down, None, 2, 1, 0)
    shape = (N, H, H, Cin)
    full, _, _ = ex._dgrad(ops, dad, csd, shape, S)                 # zero-filled, full size
    comp, _, _ = ex._dgrad(ops, dad, csd, shape, S, compact=True)   # even positions only
    assert comp.shape == (N, OHd, OHd, Cin)
    assert torch.equal(full[:, ::2, ::2], comp)
    if mode == 1:
        ref, _, _ = ex._dgrad(ops, da, cs1, shape, S, accumulate=True, dx=full.clone())
        got, _, _ = ex._dgrad(ops, da, cs1, shape, S, accumulate=True, dx=comp, sub_resid=True)
        assert torch.equal(got, ref)
        return
    # mode 4: g = (dgrad + resid)·[y > 0] with the BatchNorm-backward partials of the producer
    y = _bf(torch.randn(N, H, H, Cin, device=DEV))
    mask = torch.zeros(N * H * H * Cin // 8, dtype=torch.uint8, device=DEV)
    bits = (y.reshape(-1, 8) > 0).to(torch.uint8) << torch.arange(8, device=DEV, dtype=torch.uint8)
    mask.copy_(bits.sum(1).to(torch.uint8))
    a_prev = _bf(torch.randn(N, H, H, Cin, device=DEV))
    mi = torch.cat([torch.randn(S, Cin, device=DEV) * 0.1,
                    torch.rand(S, Cin, device=DEV) + 0.5]).reshape(-1).contiguous()
    outs = []
    for sub in (False, True):
        res = comp if sub else full.clone()
        gx, part, nb = ex._dgrad(ops, da, cs1, shape, S, dx=None if sub else res,
                                 sub_resid=sub,
                                 bn_epi=("res", res, mask, a_prev, mi, None, None))
        sums = torch.empty(2 * S * Cin, device=DEV)
        ops.bn_reduce(part, nb, S, Cin, sums)
        outs.append((gx, sums))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.allclose(outs[0][1], outs[1][1], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("N,H,Ci,Co", [(8, 16, 64, 256), (16, 8, 128, 512)])
def test_bn_backward_prologue_every_variant(ops, N, H, Ci, Co):
    """Every admissible tile variant of the 1x1 dgrad with the BN-backward operand prologue —
    the register-staged kernel and the LDS-DMA kernel (PRO 2: dY and x both DMA'd, the
    prologue applied on the landed tiles) — equals the dgrad of the materialised
    da = A·dY + B·x + D."""
    from simclr_amd.ops.conv_hip import fwd_geom  # noqa: F401  (geometry layout reference)
    torch.manual_seed(9)
    S = 2
    M = N * H * H
    g = _bf(torch.randn(N, H, H, Co, device=DEV))
    a = _bf(torch.randn(N, H, H, Co, device=DEV))
    coef = torch.randn(3 * S * Co, device=DEV) * 0.5
    wt = _bf(torch.randn(Ci, Co, device=DEV) / math.sqrt(Co)).contiguous()  # dgrad B = W^T
    da = torch.empty_like(a)
    ops.bn_bwd_apply(g, None, a, coef, S, False, da, None)
    geom = [N, H, H, Co, H, H, 1, 1, 1, 1, 1, 1, 0, 0, Ci, H, H, 1, 1, 0, 0, Ci]
    ref = torch.empty(N, H, H, Ci, device=DEV, dtype=torch.bfloat16)
    ops.igemm(da, wt, ref, None, None, geom, None, None, 0, False, 0, None, None, 0)
    c = coef.view(3, S * Co)
    seen_glds = False
    for v in range(ops.igemm_nvariants()):
        if not ops.igemm_variant_ok(v, geom, True, True) or (M // S) % ops.igemm_variant_bm(v):
            continue
        out = torch.empty_like(ref)
        ops.igemm(g, wt, out, None, None, geom, c[0], c[1], M // S, False, 0, None, None, v,
                  None, None, 0, 0, 0, None, None, None, None, None, c[2], a, None, None, None)
        assert _rel(out, ref) < 1e-2, v
        seen_glds |= ops.igemm_variant_glds(v)
    assert seen_glds, "no LDS-DMA variant admitted the BN-backward prologue"


@pytest.mark.parametrize("H,C,Co", [(32, 64, 64), (16, 128, 128)])
def test_patch_kernels_bn_apply_prologue(ops, H, C, Co):
    """The 3x3 patch kernels with the previous BatchNorm's apply + ReLU in their prologue
    (forward igemm_patch PRO 1, weight-gradient wgrad_patch PRO) == materialising
    relu(x·sc + sh) with bn_apply_ss first — every admissible variant, padding kept zero."""
    from simclr_amd.ops.conv_hip import fwd_geom
    torch.manual_seed(13)
    N, S = 8, 2
    M = N * H * H
    x = _bf(torch.randn(N, H, H, C, device=DEV))
    sc = torch.rand(S, C, device=DEV) + 0.5
    sh = torch.randn(S, C, device=DEV) * 0.5  # shifts > 0 would leak into a non-zero padding
    ss = torch.stack([sc, sh]).reshape(2, S * C).contiguous()
    xb = torch.empty_like(x)
    ops.bn_apply_ss(x, ss, None, None, xb, S, True)
    w = _bf(torch.randn(Co, 3, 3, C, device=DEV) / math.sqrt(9 * C)).contiguous()
    g = fwd_geom(N, H, H, C, H, H, 3, 3, 1, 1, Co)
    ref = torch.empty(N, H, H, Co, device=DEV, dtype=torch.bfloat16)
    ops.igemm(xb, w, ref, None, None, g, None, None, 0, False, 0, None, None, 15 if Co == 64 else 16)
    patch_seen = False
    for v in range(ops.igemm_nvariants()):
        if not ops.igemm_variant_ok(v, g, True, False) or (M // S) % ops.igemm_variant_bm(v):
            continue
        out = torch.empty_like(ref)
        ops.igemm(x, w, out, None, None, g, ss[0], ss[1], M // S, True, 0, None, None, v)
        assert _rel(out, ref) < 1e-2, v
        patch_seen |= ops.igemm_variant_glds(v)  # the only LDS-DMA kernel admitting a padded pro
    assert patch_seen
    dy = _bf(torch.randn(N, H, H, Co, device=DEV))
    outs = {}
    for v in range(ops.wgrad_nvariants()):
        if not ops.wgrad_variant_ok(v, g, True, False):
            continue
        sp = ops.wgrad_splits(g, v)
        part = torch.empty(sp * Co * 9 * C, device=DEV)
        o = torch.empty(Co, 3, 3, C, device=DEV)
        ops.wgrad(dy, x, part, o, g, sp, C, 0.0, ss[0], ss[1], M // S, True, S, v)
        outs[v] = o
    sp = ops.wgrad_splits(g, 17)
    part = torch.empty(sp * Co * 9 * C, device=DEV)
    wref = torch.empty(Co, 3, 3, C, device=DEV)
    ops.wgrad(dy, xb, part, wref, g, sp, C, 0.0, None, None, 0, False, 1, 17)
    assert 17 in outs, "wgrad_patch did not admit the X prologue"
    for v, o in outs.items():
        assert _rel(o, wref) < 1e-2, v


@pytest.mark.parametrize("splits", [1, 3])
def test_wgrad_dy_prologue_split_straddles_views(ops, splits):
    """The register-staged weight gradient with the BatchNorm-backward dY prologue, with splits
    that straddle the two views' boundary (each dY row takes its own view's coefficients), ==
    the weight gradient of the materialised da = A·dY + B·a + D (and both vs fp32); one split
    writes the output directly (partial == out, no reduction)."""
    torch.manual_seed(21)
    S, N, H, Ci, Co = 2, 16, 8, 128, 256
    M = N * H * H
    g = _bf(torch.randn(N, H, H, Co, device=DEV))
    a = _bf(torch.randn(N, H, H, Co, device=DEV))
    x = _bf(torch.randn(N, H, H, Ci, device=DEV))
    coef = torch.randn(3 * S * Co, device=DEV) * 0.5
    da = torch.empty_like(a)
    ops.bn_bwd_apply(g, None, a, coef, S, False, da, None)
    geom = [N, H, H, Ci, H, H, 1, 1, 1, 1, 1, 1, 0, 0, Co, H, H, 1, 1, 0, 0, Co]
    ref = (da.float().reshape(M, Co).t() @ x.float().reshape(M, Ci))
    seen = 0
    for v in range(ops.wgrad_nvariants()):
        if ops.wgrad_variant_glds(v) or not ops.wgrad_variant_ok(v, geom, False, True):
            continue
        out = torch.full((Co, Ci), float("nan"), device=DEV)
        part = out if splits == 1 else torch.empty(splits * Co * Ci, device=DEV)
        ops.wgrad(g, x, part, out, geom, splits, Ci, 0.0, None, None, 0, False, 1, v, a, coef,
                  M // S, S)
        assert _rel(out, ref) < 1e-2, (v, splits)
        seen += 1
    assert seen >= 2


@pytest.mark.parametrize("N,H,C", [(8, 32, 64), (8, 16, 128)])
def test_patch_bn_backward_prologue(ops, N, H, C):
    """The 3x3 dgrad with its output gradient's BatchNorm backward in the patch kernel's
    prologue (and that operand stored for the weight gradient, ``bnb_out``) vs the separate
    ``bn_bwd_apply`` pass followed by the plain dgrad: the stored operand matches the pass to
    the bf16 ulp, the input gradient and its BatchNorm partials within bf16 rounding."""
    from simclr_amd.models.fused import FusedStages, _BNState, _ConvSpec
    torch.manual_seed(4)
    S = 2
    conv = torch.nn.Conv2d(C, C, 3, 1, 1, bias=False).to(DEV)
    with torch.no_grad():
        conv.weight.copy_(_bf(torch.randn_like(conv.weight) / math.sqrt(C * 9)).float())
    g = _bf(torch.randn(N, H, H, C, device=DEV))        # masked gradient w.r.t. BN2's output
    a2 = _bf(torch.randn(N, H, H, C, device=DEV))       # conv2's pre-BN output
    coef = (torch.randn(3 * S * C, device=DEV) * 0.5).contiguous()
    a1 = _bf(torch.randn(N, H, H, C, device=DEV))       # conv2's input producer (BN1 + ReLU)
    sc = torch.rand(S, C, device=DEV) + 0.5
    sh = torch.randn(S, C, device=DEV) * 0.3
    mean = torch.randn(S, C, device=DEV) * 0.2
    inv = torch.rand(S, C, device=DEV) + 0.5
    bs = _BNState(torch.cat([mean, inv]).reshape(-1).contiguous(),
                  torch.stack([sc, sh]).reshape(2, S * C).contiguous(), 1.0)
    ex = FusedStages.__new__(FusedStages)
    ex.patch_bnb = True
    cs = _ConvSpec(conv, None, 1, 3, 1)
    assert ex._patch_bnb_ok(ops, cs, a2, S)
    da = torch.empty_like(g)
    ops.bn_bwd_apply(g, None, a2, coef, S, False, da, None)
    dx_a, part_a, nb_a = ex._dgrad(ops, da, cs, a1.shape, S, bn_epi=("mask", a1, bs))
    dy_m = torch.empty_like(g)
    dx_b, part_b, nb_b = ex._dgrad(ops, g, cs, a1.shape, S, bn_epi=("mask", a1, bs),
                                   bnb=(a2, coef), bnb_out=dy_m)
    torch.cuda.synchronize()
    # the same fp32 formula, but the two kernels' FMA contractions may round a handful of
    # values to the neighbouring bf16 (measured: 9 / 8 of 0.5 M / 0.26 M elements, 1 ulp; one
    # of them a cancellation A·g + B·a + D ~ 4e-6 of O(1) terms, 3e-8 apart in fp32)
    d = (dy_m.float() - da.float()).abs()
    ulp = torch.maximum(da.float().abs(), dy_m.float().abs()) * 2.0 ** -7
    assert int((d > 0).sum()) <= d.numel() * 1e-4 and bool((d <= ulp * 1.01 + 1e-6).all())
    assert _rel(dx_b, dx_a) < 1e-2
    sa = torch.empty(2 * S * C, device=DEV)
    sb = torch.empty(2 * S * C, device=DEV)
    ops.bn_reduce(part_a, nb_a, S, C, sa)
    ops.bn_reduce(part_b, nb_b, S, C, sb)
    assert _rel(sb, sa) < 1e-2
