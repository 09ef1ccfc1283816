"""Numerics of every hand-written HIP kernel against a plain PyTorch fp32 reference of the same op
(run on an MI355X: ``pytest -m gpu``).  Inputs are bf16-representable so the comparison isolates
the kernel's accumulation error."""
import math

import numpy as np
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


CONV_CASES = [
    # N, C, H, W, Co, k, s, p
    (4, 64, 8, 8, 64, 3, 1, 1),
    (3, 64, 9, 9, 128, 3, 2, 1),
    (2, 128, 8, 8, 256, 1, 1, 0),
    (2, 256, 8, 8, 512, 1, 2, 0),
    (5, 8, 8, 8, 64, 3, 1, 3),
    (2, 8, 16, 16, 64, 7, 2, 3),
    (1, 64, 5, 5, 64, 3, 1, 1),
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_fwd_dgrad_wgrad(ops, case):
    from simclr_amd.ops.conv_hip import ConvHipFn
    N, C, H, W, Co, k, s, p = case
    torch.manual_seed(0)
    x = _bf(torch.randn(N, C, H, W, device=DEV)).contiguous(memory_format=torch.channels_last)
    w = _bf(torch.randn(Co, C, k, k, device=DEV) / math.sqrt(C * k * k)).float()
    x.requires_grad_(True)
    wp = w.clone().requires_grad_(True)
    y = ConvHipFn.apply(x, wp, s, p, False)
    xr = x.detach().float().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, None, s, p)
    assert y.shape == yr.shape
    assert _rel(y, yr) < 1e-2
    gy = _bf(torch.randn_like(yr))
    y.backward(gy.contiguous(memory_format=torch.channels_last))
    yr.backward(gy.float())
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(wp.grad, wr.grad) < 1e-2


def test_conv_stats_epilogue(ops):
    from simclr_amd.ops.conv_hip import ConvHipFn
    torch.manual_seed(1)
    x = _bf(torch.randn(8, 64, 16, 16, device=DEV)).contiguous(memory_format=torch.channels_last)
    w = _bf(torch.randn(64, 64, 3, 3, device=DEV) / 24).float()
    y = ConvHipFn.apply(x, w, 1, 1, True)
    stats, nblk = y._simclr_stats
    st = stats.view(nblk, 2, 64)
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, 64)
    assert torch.allclose(st[:, 0].sum(0), yf.sum(0), rtol=1e-3, atol=1e-2)
    assert torch.allclose(st[:, 1].sum(0), (yf * yf).sum(0), rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("C,relu,res,S,spatial", [(64, True, False, 2, 8), (256, True, True, 2, 4),
                                                  (128, False, False, 1, 3), (2048, True, False, 2, 1)])
def test_batchnorm_train(ops, C, relu, res, S, spatial):
    from simclr_amd.ops.batchnorm import BatchNorm2d, reference_batch_norm_train
    from simclr_amd.ops.batchnorm_hip import batch_norm_train
    from simclr_amd.parallel import state as pstate
    torch.manual_seed(2)
    N = 8
    bn = BatchNorm2d(C).to(DEV)
    with torch.no_grad():
        bn.weight.copy_(torch.rand(C) + 0.5)
        bn.bias.copy_(torch.randn(C) * 0.1)
    bn_ref = BatchNorm2d(C).to(DEV)
    bn_ref.load_state_dict(bn.state_dict())
    x = _bf(torch.randn(N, C, spatial, spatial, device=DEV) * 2 + 0.5).contiguous(
        memory_format=torch.channels_last).requires_grad_(True)
    r = (_bf(torch.randn(N, C, spatial, spatial, device=DEV)).contiguous(
        memory_format=torch.channels_last).requires_grad_(True) if res else None)
    y = batch_norm_train(x, bn, S, r, relu, pstate.get())
    xr = x.detach().float().requires_grad_(True)
    rr = r.detach().float().requires_grad_(True) if res else None
    yr = reference_batch_norm_train(xr, bn_ref, S, rr, relu)
    assert _rel(y, yr) < 2e-2
    assert torch.allclose(bn.running_mean, bn_ref.running_mean, atol=1e-3, rtol=1e-3)
    assert torch.allclose(bn.running_var, bn_ref.running_var, atol=1e-3, rtol=1e-3)
    assert int(bn.num_batches_tracked) == int(bn_ref.num_batches_tracked) == S
    gy = _bf(torch.randn_like(yr))
    y.backward(gy.contiguous(memory_format=torch.channels_last))
    yr.backward(gy.float())
    assert _rel(x.grad, xr.grad) < 3e-2
    assert _rel(bn.weight.grad, bn_ref.weight.grad) < 2e-2
    assert _rel(bn.bias.grad, bn_ref.bias.grad) < 2e-2
    if res:
        assert _rel(r.grad, rr.grad) < 2e-2


def test_avgpool(ops):
    from simclr_amd.ops.pooling_hip import AvgPoolHipFn
    x = _bf(torch.randn(6, 64, 4, 4, device=DEV)).contiguous(
        memory_format=torch.channels_last).requires_grad_(True)
    y = AvgPoolHipFn.apply(x)
    xr = x.detach().float().requires_grad_(True)
    yr = xr.mean(dim=(2, 3))
    assert _rel(y, yr) < 1e-2
    g = _bf(torch.randn(6, 64, device=DEV))
    y.backward(g)
    yr.backward(g.float())
    assert _rel(x.grad, xr.grad) < 1e-2


def test_linear(ops):
    from simclr_amd.ops.gemm_hip import LinearHipFn
    torch.manual_seed(3)
    x = _bf(torch.randn(256, 512, device=DEV)).requires_grad_(True)
    w = _bf(torch.randn(128, 512, device=DEV) / 22).float().requires_grad_(True)
    b = torch.randn(128, device=DEV).requires_grad_(True)
    y = LinearHipFn.apply(x, w, b, False)
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().clone().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    yr = F.linear(xr, wr, br)
    assert _rel(y, yr) < 1e-2
    g = _bf(torch.randn(256, 128, device=DEV))
    y.backward(g)
    yr.backward(g.float())
    assert _rel(x.grad, xr.grad) < 1e-2
    assert _rel(w.grad, wr.grad) < 1e-2
    assert _rel(b.grad, br.grad) < 1e-2


@pytest.mark.parametrize("n,d,tau", [(64, 128, 0.5), (512, 128, 0.5), (32, 64, 0.1)])
def test_ntxent(ops, n, d, tau):
    from simclr_amd.loss.ntxent import NTXent, nt_xent_torch
    torch.manual_seed(4)
    z = _bf(torch.randn(2 * n, d, device=DEV)).requires_grad_(True)
    loss = NTXent(tau)(z)
    zr = z.detach().float().requires_grad_(True)
    lr = nt_xent_torch(zr, n, tau)
    assert abs(loss.item() - lr.item()) < 1e-4 * max(1.0, abs(lr.item()))
    loss.backward()
    lr.backward()
    assert _rel(z.grad, zr.grad) < 1e-2


def test_ntxent_matches_reference_formulation(ops):
    """HIP NT-Xent == the reference's mask/concat formulation (loss.py:33-65)."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
    from bench.torch_reference import nt_xent_reference
    from simclr_amd.loss.ntxent import NTXent
    torch.manual_seed(5)
    v0 = _bf(torch.randn(128, 128, device=DEV))
    v1 = _bf(torch.randn(128, 128, device=DEV))
    a = NTXent(0.5)(v0, v1).item()
    b = nt_xent_reference(v0.float(), v1.float(), 0.5).item()
    assert abs(a - b) < 1e-4


def test_lars_kernel_matches_torch(ops):
    from simclr_amd.models import ContrastiveModel
    from simclr_amd.optim.lars import FusedLARS, weight_decay_per_param
    from simclr_amd.parallel.flat import FlatParamStore
    from simclr_amd.ops import registry
    torch.manual_seed(6)
    stores = []
    for _ in range(2):
        torch.manual_seed(6)
        m = ContrastiveModel("resnet18").to(DEV)
        st = FlatParamStore(m, DEV, shadow_dtype=torch.bfloat16)
        stores.append(st)
    g = torch.randn(stores[0].total, device=DEV) * 1e-2
    for st in stores:
        st.grad.copy_(g)
    opts = [FusedLARS(st, weight_decay_per_param(st, 1e-4), lr0=2.0, warmup_steps=3,
                      total_steps=20) for st in stores]
    for _ in range(5):
        opts[0].step()
        registry.set_backend("torch")
        try:
            opts[1].step()
        finally:
            registry.set_backend("auto")
    assert torch.allclose(stores[0].master, stores[1].master, rtol=1e-5, atol=1e-6)
    assert torch.allclose(opts[0].mom, opts[1].mom, rtol=1e-4, atol=1e-6)
    assert torch.equal(stores[0].shadow, stores[0].master.to(torch.bfloat16))
    assert abs(opts[0].lr_t.item() - opts[1].lr_t.item()) < 1e-6


@pytest.mark.parametrize("n,splits,beta", [(4096, 32, 0.0), (16384, 257, 0.0), (65536, 100, 1.0),
                                           (65536, 31, 0.0), (262144, 64, 0.0)])
def test_wgrad_reduce_slabs_matches_sum(ops, n, splits, beta):
    """Split-slab reduction (the column-parallel single launch for small outputs with >= 32
    splits, the two-level one otherwise) vs an fp64 sum; deterministic across launches."""
    torch.manual_seed(n + splits)
    part = torch.randn(splits * n, device=DEV)
    out0 = torch.randn(n, device=DEV)
    ref = part.view(splits, n).double().sum(0) + beta * out0.double()
    got = []
    for _ in range(2):
        out = out0.clone()
        ops.wgrad_reduce_slabs(part.clone(), splits, out, beta)
        got.append(out)
    torch.cuda.synchronize()
    assert torch.equal(got[0], got[1])
    assert float((got[0].double() - ref).abs().max()) < 1e-4 * math.sqrt(splits)


def test_lars_early_groups_bitwise(ops):
    """The optimizer update split into early groups (issued out of order, on another stream)
    plus the rest in step() equals the single whole-store update bitwise: same chunks, same
    per-segment reduction order."""
    from simclr_amd.models import ContrastiveModel
    from simclr_amd.optim.lars import FusedLARS, weight_decay_per_param
    from simclr_amd.parallel.flat import FlatParamStore
    stores = []
    for _ in range(2):
        torch.manual_seed(7)
        m = ContrastiveModel("resnet18").to(DEV)
        stores.append(FlatParamStore(m, DEV, shadow_dtype=torch.bfloat16))
    opts = [FusedLARS(st, weight_decay_per_param(st, 1e-4), lr0=2.0, warmup_steps=3,
                      total_steps=20) for st in stores]
    names = stores[1].names
    groups = {4: [i for i, n in enumerate(names) if ".layer4." in n or n.startswith("g.")],
              3: [i for i, n in enumerate(names) if ".layer3." in n]}
    opts[1].set_early_groups(groups)
    side = torch.cuda.Stream(device=DEV)
    for k in range(5):
        g = torch.randn(stores[0].total, device=DEV) * 1e-2
        for st in stores:
            st.grad.copy_(g)
        opts[0].step()
        side.wait_stream(torch.cuda.current_stream(DEV))
        with torch.cuda.stream(side):
            opts[1].early_step(3)
            if k % 2:
                opts[1].early_step(4)  # odd steps: group 4 issued early, else left to step()
        torch.cuda.current_stream(DEV).wait_stream(side)
        opts[1].step()
    torch.cuda.synchronize()
    assert torch.equal(stores[0].master, stores[1].master)
    assert torch.equal(opts[0].mom, opts[1].mom)
    assert torch.equal(stores[0].shadow, stores[1].shadow)
    assert torch.equal(opts[0].lr_t, opts[1].lr_t) and torch.equal(opts[0].step_t, opts[1].step_t)


def test_augment_matches_numpy(ops):
    from simclr_amd.data import augment_ref
    rng = np.random.default_rng(0)
    imgs = rng.integers(0, 256, size=(16, 32, 32, 3), dtype=np.uint8)
    idx = np.arange(16, dtype=np.int64)
    n, views = 16, 2
    out = torch.empty((views * n, 32, 32, 8), device=DEV, dtype=torch.bfloat16)
    params = torch.empty((views * n * 16,), device=DEV, dtype=torch.float32)
    ops.augment(torch.from_numpy(imgs).to(DEV), torch.from_numpy(idx).to(DEV), n, views, 32, 32, 8,
                0.5, 7, 3, 0, 1, out, params)
    ref = augment_ref.augment_batch(imgs, idx, views, 32, 32, 0.5, 7, 3)
    got = out.float().cpu().numpy()[..., :3].transpose(0, 3, 1, 2)
    assert (out.float()[..., 3:] == 0).all()
    diff = np.abs(got - ref)
    # bf16 output quantisation + float transcendental differences: almost all pixels equal
    assert np.mean(diff < 2.5 / 255 + 4e-3) > 0.97
    # and the sampled parameters agree for (nearly) every image
    P = params.view(views * n, 16).cpu().numpy()
    same = 0
    for v in range(views):
        for b in range(n):
            p = augment_ref.sample_params(
                augment_ref.Rng(augment_ref.image_key(7, 3, v, b)), 32, 32, 0.5)
            row = P[v * n + b]
            same += int(row[0] == p["ci"] and row[1] == p["cj"] and row[2] == p["ch"]
                        and row[3] == p["cw"] and bool(row[4]) == p["flip"])
    assert same >= views * n - 1


def test_augment_large_matches_numpy(ops):
    """Outputs above 64x64 (ImageNet shape, BASELINE config 5) take the two-pass kernel."""
    from simclr_amd.data import augment_ref
    rng = np.random.default_rng(3)
    S = 80
    imgs = rng.integers(0, 256, size=(8, S, S, 3), dtype=np.uint8)
    idx = np.arange(8, dtype=np.int64)
    n, views = 8, 2
    out = torch.empty((views * n, S, S, 8), device=DEV, dtype=torch.bfloat16)
    ops.augment(torch.from_numpy(imgs).to(DEV), torch.from_numpy(idx).to(DEV), n, views, S, S, 8,
                0.5, 7, 3, 0, 1, out, None)
    ref = augment_ref.augment_batch(imgs, idx, views, S, S, 0.5, 7, 3)
    got = out.float().cpu().numpy()[..., :3].transpose(0, 3, 1, 2)
    assert np.mean(np.abs(got - ref) < 2.5 / 255 + 4e-3) > 0.97


def test_augment_plain_mode(ops):
    rng = np.random.default_rng(1)
    imgs = torch.from_numpy(rng.integers(0, 256, size=(4, 32, 32, 3), dtype=np.uint8)).to(DEV)
    out = torch.empty((4, 32, 32, 8), device=DEV, dtype=torch.bfloat16)
    ops.augment(imgs, None, 4, 1, 32, 32, 8, 0.5, 0, 0, 0, 0, out, None)
    ref = imgs.float() / 255
    assert torch.allclose(out.float()[..., :3], ref, atol=4e-3)


@pytest.mark.parametrize("k,s,p", [(1, 1, 0), (3, 1, 1), (3, 2, 1)])
def test_igemm_variants_prologue_epilogue(ops, k, s, p):
    """Every tile variant, with the fused BN-apply prologue and both epilogue modes, against an
    fp32 torch reference; and the wgrad kernel variants with the prologue."""
    from simclr_amd.ops.conv_hip import fwd_geom
    torch.manual_seed(7)
    N, C, H, W, Co = 8, 64, 16, 16, 128
    S = 2
    x = _bf(torch.randn(N, C, H, W, device=DEV))
    sc = (torch.rand(S, C, device=DEV) + 0.5).contiguous()
    sh = (torch.randn(S, C, device=DEV) * 0.3).contiguous()
    seg = torch.arange(N, device=DEV) // (N // S)
    a = torch.relu(x.float() * sc[seg][:, :, None, None] + sh[seg][:, :, None, None])
    a = _bf(a).float()
    w = _bf(torch.randn(Co, C, k, k, device=DEV) / (C * k * k) ** 0.5)
    ref = F.conv2d(a, w.float(), None, s, p)
    OH, OW = ref.shape[-2:]
    M = N * OH * OW
    g = fwd_geom(N, H, W, C, OH, OW, k, k, s, p, Co)
    xn = x.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1)
    wo = w.permute(0, 2, 3, 1).contiguous()
    r = _bf(torch.randn(N, OH, OW, Co, device=DEV))
    yy = _bf(torch.randn(N, OH, OW, Co, device=DEV))
    refn = ref.permute(0, 2, 3, 1)
    for v in range(ops.igemm_nvariants()):
        bm = ops.igemm_variant_bm(v)
        if (M // S) % bm or not ops.igemm_variant_ok(v, g, True, False):
            continue
        out = torch.empty(N, OH, OW, Co, device=DEV, dtype=torch.bfloat16)
        ops.igemm(xn, wo, out, None, None, g, sc, sh, M // S, True, 0, None, None, v)
        assert _rel(out, refn) < 1e-2, v
        ops.igemm(xn, wo, out, None, None, g, sc, sh, M // S, True, 1, r, None, v)
        assert _rel(out, refn + r.float()) < 1e-2, v
        ops.igemm(xn, wo, out, None, None, g, sc, sh, M // S, True, 2, r, yy, v)
        assert _rel(out, refn + torch.where(yy.float() > 0, r.float(), 0.0)) < 1e-2, v
    # wgrad with the same prologue
    wr = w.float().clone().requires_grad_(True)
    yref = F.conv2d(a, wr, None, s, p)
    gy = _bf(torch.randn_like(yref))
    yref.backward(gy.float())
    dyn = gy.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1)
    for v in range(ops.wgrad_nvariants()):
        if not ops.wgrad_variant_ok(v, g, True, False):
            continue
        splits = ops.wgrad_splits(g, v)
        K = k * k * C
        part = torch.empty(splits * Co * K, device=DEV)
        out = torch.empty(Co, k, k, C, device=DEV)
        ops.wgrad(dyn, xn, part, out, g, splits, C, 0.0, sc, sh, M // S, True, S, v)
        assert _rel(out.permute(0, 3, 1, 2), wr.grad) < 1e-2, v


@pytest.mark.parametrize("C,Co,H,affine_res", [(256, 64, 16, False), (256, 64, 16, True),
                                               (512, 128, 8, True), (1024, 256, 4, False),
                                               (2048, 512, 4, False)])
def test_igemm_block_output_prologue(ops, C, Co, H, affine_res):
    """conv1 of the next block forming the block output in its prologue == bn_apply_ss (block
    output + ReLU mask) followed by the plain conv: out, mask and the BN statistics partials,
    for every admissible tile (identity and downsample-BN residuals, one or two N tiles)."""
    from simclr_amd.ops.conv_hip import fwd_geom
    torch.manual_seed(C + Co)
    S, N = 2, 16
    R = N * H * H
    aL = _bf(torch.randn(R, C, device=DEV))
    res = _bf(torch.randn(R, C, device=DEV))
    ss = torch.stack([torch.rand(S, C, device=DEV) + 0.5,
                      torch.randn(S, C, device=DEV) * 0.3]).contiguous()
    rss = (torch.stack([torch.rand(S, C, device=DEV) + 0.5, torch.randn(S, C, device=DEV)])
           .contiguous() if affine_res else None)
    w = _bf(torch.randn(Co, C, device=DEV) / C ** 0.5)
    g = fwd_geom(N, H, H, C, H, H, 1, 1, 1, 0, Co)
    out_ref = torch.empty_like(aL)
    mask_ref = torch.empty(R * C // 8, device=DEV, dtype=torch.uint8)
    ops.bn_apply_ss(aL, ss.view(-1), res, None if rss is None else rss.view(-1), out_ref, S, True,
                    mask_ref)
    vs = [v for v in range(ops.igemm_nvariants())
          if ops.igemm_dual_ok(v, g) and (R // S) % ops.igemm_variant_bm(v) == 0]
    assert vs, "no tile admits the block-output prologue"
    ref = out_ref.float() @ w.float().t()
    for v in vs:
        bm = ops.igemm_variant_bm(v)
        y0 = torch.empty(R, Co, device=DEV, dtype=torch.bfloat16)
        st0 = torch.empty((R // bm) * 2 * Co, device=DEV)
        ops.igemm(out_ref, w, y0, None, st0, g, variant=v)
        out = torch.full_like(aL, float("nan"))
        mask = torch.zeros_like(mask_ref)
        y1 = torch.empty_like(y0)
        st1 = torch.empty_like(st0)
        ops.igemm(aL, w, y1, None, st1, g, ss[0].reshape(-1), ss[1].reshape(-1), R // S, True,
                  variant=v, A2=res, pro_rss=None if rss is None else rss.view(-1), pro_out=out,
                  pro_mask=mask)
        torch.cuda.synchronize()
        d = (out.float() - out_ref.float()).abs()
        assert d.max().item() <= 1e-2 * out_ref.float().abs().max().item(), v
        same = (out == out_ref).view(-1, 8).all(1)  # bytes whose 8 outputs agree bit-exactly
        assert torch.equal(mask[same], mask_ref[same]), v
        assert same.float().mean().item() > 0.99, v
        assert _rel(y1, ref) < 1e-2 and _rel(y1, y0) < 1e-2, v
        assert _rel(st1, st0) < 1e-2, v


def _glds_variants(ops):
    return [v for v in range(ops.igemm_nvariants()) if ops.igemm_variant_glds(v)]


@pytest.mark.parametrize("k,s,p,C,Co,H", [(1, 1, 0, 64, 256, 16), (3, 1, 1, 64, 64, 16),
                                           (3, 2, 1, 128, 192, 16), (1, 2, 0, 128, 128, 16),
                                           (3, 1, 1, 128, 512, 16), (3, 1, 1, 64, 64, 32),
                                           (3, 1, 1, 128, 128, 32)])
def test_igemm_glds_variants(ops, k, s, p, C, Co, H):
    """The LDS-DMA kernel (igemm_glds): every tile variant against an fp32 torch conv (plain,
    +residual, masked residual, BN statistics partials) and against the register-staged kernel
    for the BatchNorm-backward epilogues (modes 3 and 4, per-segment tables)."""
    from simclr_amd.ops.conv_hip import fwd_geom
    torch.manual_seed(11)
    N, W, S = 8, H, 2
    x = _bf(torch.randn(N, C, H, W, device=DEV))
    w = _bf(torch.randn(Co, C, k, k, device=DEV) / (C * k * k) ** 0.5)
    ref = F.conv2d(x.float(), w.float(), None, s, p)
    OH, OW = ref.shape[-2:]
    M = N * OH * OW
    g = fwd_geom(N, H, W, C, OH, OW, k, k, s, p, Co)
    xn = x.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1)
    wo = w.permute(0, 2, 3, 1).contiguous()
    refn = ref.permute(0, 2, 3, 1)
    r = _bf(torch.randn(N, OH, OW, Co, device=DEV))
    yy = _bf(torch.randn(N, OH, OW, Co, device=DEV))
    xa = _bf(torch.randn(N, OH, OW, Co, device=DEV))
    mi = torch.cat([torch.randn(S, Co, device=DEV) * 0.2,
                    torch.rand(S, Co, device=DEV) + 0.5]).reshape(-1).contiguous()
    ss = torch.cat([torch.rand(S, Co, device=DEV) + 0.5,
                    torch.randn(S, Co, device=DEV) * 0.3]).reshape(-1).contiguous()
    seg = M // S
    vs = _glds_variants(ops)
    assert vs
    base_v = 0

    def run(v, mode, stats=False, **kw):
        bm = ops.igemm_variant_bm(v)
        out = torch.empty(N, OH, OW, Co, device=DEV, dtype=torch.bfloat16)
        st = torch.empty((M // bm) * 2 * Co, device=DEV) if stats else None
        ea = kw.get("ea")
        eb = kw.get("eb")
        ops.igemm(xn, wo, out, None, st, g, None, None, 0, False, mode, ea, eb, v,
                  kw.get("ess"), kw.get("emi"), seg if mode >= 3 else 0, 0, 0, kw.get("ec"),
                  None, None, None, None, None, None)
        return out, (st.view(M // bm, 2, Co).sum(0) if stats else None)

    for v in vs:
        if seg % ops.igemm_variant_bm(v) or not ops.igemm_variant_ok(v, g, False, False):
            continue
        out, st = run(v, 0, stats=True)
        assert _rel(out, refn) < 1e-2, v
        of = out.float().reshape(-1, Co)
        assert _rel(st[0], of.sum(0)) < 1e-3 and _rel(st[1], (of * of).sum(0)) < 1e-3, v
        out, _ = run(v, 1, ea=r)
        assert _rel(out, refn + r.float()) < 1e-2, v
        out, _ = run(v, 2, ea=r, eb=yy)
        assert _rel(out, refn + torch.where(yy.float() > 0, r.float(), 0.0)) < 1e-2, v
        for mode, kw in ((3, dict(eb=yy, ess=ss, emi=mi)), (4, dict(ea=r, eb=yy, ec=xa, emi=mi))):
            out, st = run(v, mode, stats=True, **kw)
            o0, s0 = run(base_v, mode, stats=True, **kw)
            assert _rel(out, o0) < 1e-2, (v, mode)
            assert _rel(st, s0) < 1e-3, (v, mode)


@pytest.mark.parametrize("k,s,p,C,Co,H", [(1, 1, 0, 64, 256, 16), (3, 1, 1, 64, 64, 16),
                                           (3, 2, 1, 128, 192, 16), (1, 2, 0, 128, 128, 16),
                                           (3, 1, 1, 256, 512, 4), (3, 1, 1, 64, 64, 5),
                                           (3, 1, 1, 64, 64, 32), (3, 1, 1, 128, 128, 16),
                                           (3, 1, 1, 128, 64, 32), (3, 1, 1, 64, 128, 8),
                                           (3, 2, 1, 64, 64, 8)])
@pytest.mark.parametrize("xlin", [0, 1])
def test_wgrad_glds_variants(ops, k, s, p, C, Co, H, xlin):
    """LDS-DMA weight gradient (wgrad_glds), every tile variant and a few split counts, against
    torch's fp32 conv2d weight gradient (partial M tiles: H=5 gives M % 64 != 0).  The 1x1
    stride-1 cases and the ones with OH * OW dividing 64 (8x8, 4x4 outputs) run wgrad_xp's
    step-affine X addressing (XLIN)."""
    from simclr_amd.ops.conv_hip import fwd_geom
    torch.manual_seed(13)
    N = 8
    x = _bf(torch.randn(N, C, H, H, device=DEV))
    wr = (_bf(torch.randn(Co, C, k, k, device=DEV)) * 0.05).float().requires_grad_(True)
    y = F.conv2d(x.float(), wr, None, s, p)
    gy = _bf(torch.randn_like(y))
    y.backward(gy.float())
    OH, OW = y.shape[-2:]
    g = fwd_geom(N, H, H, C, OH, OW, k, k, s, p, Co)
    xn = x.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1)
    dyn = gy.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1)
    K = k * k * C
    vs = [v for v in range(ops.wgrad_nvariants())
          if ops.wgrad_variant_glds(v) and ops.wgrad_variant_ok(v, g, False, False)]
    assert vs
    prev = ops.wgrad_xlin(-1)
    assert ops.wgrad_xlin(xlin) == xlin
    try:
        for v in vs:
            base = ops.wgrad_splits(g, v)
            for splits in sorted({1, 3, base}):
                part = torch.empty(splits * Co * K, device=DEV)
                out = torch.empty(Co, k, k, C, device=DEV)
                ops.wgrad(dyn, xn, part, out, g, splits, C, 0.0, None, None, 0, False, 1, v)
                assert _rel(out.permute(0, 3, 1, 2), wr.grad) < 1e-2, (v, splits)
    finally:
        ops.wgrad_xlin(prev)


@pytest.mark.parametrize("k,p,C,Co,H", [(3, 1, 128, 128, 16), (3, 1, 64, 128, 32),
                                        (1, 0, 128, 256, 16), (3, 1, 256, 256, 8)])
def test_igemm_dgrad_parity_classes_every_variant(ops, k, p, C, Co, H):
    """Stride-2 input gradient as parity-class sub-convolutions (negative tap step, strided
    output rows — the geometry models/fused.py ``_dgrad`` builds): every admissible tile variant,
    register-staged and LDS-DMA, writes exactly its class's positions and matches fp32
    ``conv2d_input`` there."""
    from simclr_amd.models.fused import FusedStages, _ConvSpec
    torch.manual_seed(17)
    N, s = 8, 2
    w = _bf(torch.randn(Co, C, k, k, device=DEV) / (C * k * k) ** 0.5)
    OH = (H + 2 * p - k) // s + 1
    dy = _bf(torch.randn(N, Co, OH, OH, device=DEV))
    ref = torch.nn.grad.conv2d_input((N, C, H, H), w.float(), dy.float(), s, p).permute(0, 2, 3, 1)
    dyn = dy.permute(0, 2, 3, 1).contiguous()
    wo = w.permute(0, 2, 3, 1).contiguous()
    cs = _ConvSpec(torch.nn.Conv2d(C, Co, k, s, p, bias=False), None, s, k, p)
    covered = torch.zeros(H, H, dtype=torch.bool, device=DEV)
    seen_glds = False
    for (r, c), prm in FusedStages._wt_params(cs):
        wt = torch.empty((prm[3], prm[4], prm[5], prm[0]), device=DEV, dtype=torch.bfloat16)
        ops.weight_transform(wo, wt, prm)
        _, _, _, _, nkh, nkw, kh0, _, kw0, _ = prm
        ohc, owc = (H - r + 1) // 2, (H - c + 1) // 2
        g = [N, OH, OH, Co, ohc, owc, nkh, nkw, 1, 1, -1, -1, (r + p - kh0) // 2,
             (c + p - kw0) // 2, C, H, H, 2, 2, r, c, C]
        M = N * ohc * owc
        n_ok = 0
        for v in range(ops.igemm_nvariants()):
            if not ops.igemm_variant_ok(v, g, False, False) or M % ops.igemm_variant_bm(v):
                continue
            dx = torch.full((N, H, H, C), float("nan"), device=DEV, dtype=torch.bfloat16)
            ops.igemm(dyn, wt, dx, None, None, g, None, None, 0, False, 0, None, None, v,
                      None, None, 0, 0, 0, None, None, None, None, None, None, None)
            cls = dx[:, r::2, c::2]
            assert _rel(cls, ref[:, r::2, c::2]) < 1e-2, (v, r, c)
            mask = torch.ones(H, H, dtype=torch.bool, device=DEV)
            mask[r::2, c::2] = False
            assert bool(torch.isnan(dx[:, mask].float()).all()), ("wrote outside its class", v)
            seen_glds |= ops.igemm_variant_glds(v)
            n_ok += 1
        assert n_ok >= 2, (r, c)
        covered[r::2, c::2] = True
    assert bool(covered.all()) or k == 1
    assert seen_glds, "no LDS-DMA variant admitted the parity-class geometry"


@pytest.mark.parametrize("k,s,p,H", [(3, 1, 1, 32), (3, 1, 3, 32)])
def test_wgrad_bn_backward_prologue_padded_channels(ops, k, s, p, H):
    """The stem's weight gradient as the fused executor runs it: the dY operand is the
    BatchNorm backward A·dY + B·Y + D of the stem's own BN (per-row view segment, computed in
    the prologue), the input holds 3 real image channels gathered as 8, and the result is
    compacted to the 3 real channels (in-place slab sum, then compaction).  Every admissible
    variant, with split counts aligned to the views and — for the register-staged variants,
    which take each row's own segment — counts that straddle the view boundary, against torch's
    fp32 conv2d weight gradient of the same operands."""
    from simclr_amd.ops.conv_hip import fwd_geom, run_wgrad
    torch.manual_seed(17)
    N, C, Creal, Co, S = 16, 8, 3, 64, 2
    x = _bf(torch.randn(N, C, H, H, device=DEV))
    y = F.conv2d(x.float()[:, :Creal], torch.randn(Co, Creal, k, k, device=DEV) * 0.3, None, s, p)
    Y = _bf(y)  # the BN input (pre-BN conv output), stored bf16
    gy = _bf(torch.randn_like(y))
    OH, OW = y.shape[-2:]
    M = N * OH * OW
    seg = M // S
    coef = torch.cat([torch.rand(S, Co, device=DEV) + 0.5, torch.randn(S, Co, device=DEV) * 0.2,
                      torch.randn(S, Co, device=DEV) * 0.1]).reshape(-1).contiguous()
    A, B, D = coef.view(3, S, Co)
    segi = torch.arange(N, device=DEV) // (N // S)
    dy_eff = (A[segi][:, :, None, None] * gy.float() + B[segi][:, :, None, None] * Y.float()
              + D[segi][:, :, None, None])
    wr = torch.zeros(Co, Creal, k, k, device=DEV, requires_grad=True)
    F.conv2d(x.float()[:, :Creal], wr, None, s, p).backward(dy_eff)
    ref = wr.grad
    g = fwd_geom(N, H, H, C, OH, OW, k, k, s, p, Co)
    xn = x.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1)
    dyn = gy.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1)
    Yn = Y.contiguous(memory_format=torch.channels_last).permute(0, 2, 3, 1)
    K = k * k * C
    vs = [v for v in range(ops.wgrad_nvariants()) if ops.wgrad_variant_ok(v, g, False, True)]
    assert vs
    checked = 0
    for v in vs:
        cands = {S, 2 * S, S * max(1, ops.wgrad_splits(g, v) // S)}
        if not ops.wgrad_variant_glds(v):
            cands |= {1, 3}  # straddling the view boundary
        for splits in sorted(cands):
            if splits > 1 and (M // 64) < splits:
                continue
            part = torch.full((splits * Co * K,), float("nan"), device=DEV)
            out = torch.full((Co, k, k, Creal), float("nan"), device=DEV)
            ops.wgrad(dyn, xn, part, out, g, splits, Creal, 0.0, None, None, 0, False, 1, v,
                      Yn, coef, seg, S)
            torch.cuda.synchronize()
            assert _rel(out.permute(0, 3, 1, 2), ref) < 1e-2, (v, splits)
            checked += 1
    # the production entry point (autotuned variant, aligned splits)
    out = torch.empty(Co, k, k, Creal, device=DEV)
    run_wgrad(ops, dyn, xn, out, g, Creal, dpro=(Yn, coef, seg, S))
    assert _rel(out.permute(0, 3, 1, 2), ref) < 1e-2
    assert checked >= len(vs)


@pytest.mark.parametrize("N,H,creal", [(2, 224, 3), (4, 32, 3), (3, 30, 2)])
def test_stem_s2d_kernel(ops, N, H, creal):
    """k_stem_s2d: the padded image's 2x2 space-to-depth, bitwise equal to the torch reshuffle
    (channels >= creal zeroed even where the image holds garbage there)."""
    from test_stem_s2d import s2d_reference
    torch.manual_seed(5)
    img = _bf(torch.randn(N, H, H, 8, device=DEV))
    xs = torch.full((N, (H + 6) // 2, (H + 6) // 2, 16), 7.0, device=DEV, dtype=torch.bfloat16)
    ops.stem_s2d(img, creal, 3, xs)
    torch.cuda.synchronize()
    assert torch.equal(xs, s2d_reference(img, creal))


@pytest.mark.parametrize("N,H,C", [(4, 16, 64), (6, 17, 64), (2, 112, 64)])
def test_pooled_stem_kernels(ops, N, H, C):
    """The ImageNet stem's fused BN + ReLU + MaxPool2d(3, 2, 1) forward (bn_relu_maxpool) and
    max-pool / ReLU-mask / BN input-gradient backward (maxpool_bwd_bn) against fp32 torch on the
    same bf16 operands: pooled values, the recorded argmax / pre-BN value, and
    da = A·g + B·a + D with g = max-pool backward of the pooled gradient masked by [pooled > 0]
    (odd H: windows clipped at the border)."""
    torch.manual_seed(N * H + C)
    S, K, Sd, P = 2, 3, 2, 1
    a = _bf(torch.randn(N, H, H, C, device=DEV))
    ss = torch.cat([torch.rand(S, C, device=DEV) + 0.5,
                    torch.randn(S, C, device=DEV) * 0.5]).reshape(-1).contiguous()
    OH = (H + 2 * P - K) // Sd + 1
    y = torch.empty(N, OH, OH, C, device=DEV, dtype=torch.bfloat16)
    arg = torch.empty(y.shape, device=DEV, dtype=torch.uint8)
    asel = torch.empty_like(y)
    ops.bn_relu_maxpool(a, ss, S, y, arg, asel, K, Sd, P)
    seg = torch.arange(N, device=DEV) // (N // S)
    sc = ss[:S * C].view(S, C)[seg][:, None, None, :]
    sh = ss[S * C:].view(S, C)[seg][:, None, None, :]
    r = _bf(torch.relu(torch.addcmul(sh, a.float(), sc))).float()  # what a BN-apply pass stores
    ref, idx = F.max_pool2d(r.permute(0, 3, 1, 2), K, Sd, P, return_indices=True)
    # (torch may round the affine differently from the kernel's fma in the last fp32 bit,
    # which can flip a bf16 rounding now and then)
    assert (y.float() != ref.permute(0, 2, 3, 1)).float().mean().item() < 1e-3
    assert _rel(y, ref.permute(0, 2, 3, 1)) < 1e-2
    # the recorded tap points at a window element holding the maximum, and asel is its a
    t = arg.long()
    ih = torch.arange(OH, device=DEV)[None, :, None, None] * Sd - P + t // K
    iw = torch.arange(OH, device=DEV)[None, None, :, None] * Sd - P + t % K
    n_ = torch.arange(N, device=DEV)[:, None, None, None]
    c_ = torch.arange(C, device=DEV)[None, None, None, :]
    assert (r[n_, ih, iw, c_] != y.float()).float().mean().item() < 1e-3
    assert torch.equal(a[n_, ih, iw, c_], asel)
    # backward
    gy = _bf(torch.randn_like(y.float()))
    coef = torch.cat([torch.rand(S, C, device=DEV) + 0.5, torch.randn(S, C, device=DEV) * 0.2,
                      torch.randn(S, C, device=DEV) * 0.1]).reshape(-1).contiguous()
    da = torch.empty_like(a)
    ops.maxpool_bwd_bn(gy, arg, y, a, coef, S, da, K, Sd, P)
    flat = ((n_ * H + ih) * H + iw) * C + c_
    g = torch.zeros(N * H * H * C, device=DEV)
    g.index_add_(0, flat.reshape(-1), (gy.float() * (y.float() > 0)).reshape(-1))
    g = g.view(N, H, H, C)
    A = coef[:S * C].view(S, C)[seg][:, None, None, :]
    B = coef[S * C:2 * S * C].view(S, C)[seg][:, None, None, :]
    D = coef[2 * S * C:].view(S, C)[seg][:, None, None, :]
    dref = A * g + B * a.float() + D
    assert _rel(da, dref) < 1e-2
    # the BatchNorm-backward partials from pooled-size tensors equal the full-resolution sums
    mi = torch.cat([torch.randn(S, C, device=DEV) * 0.1,
                    torch.rand(S, C, device=DEV) + 0.5]).reshape(-1).contiguous()
    nblk = ops.bn_blocks(y.numel() // C, C, S)
    part = torch.empty(S * nblk * 2 * C, device=DEV)
    ops.bn_bwd_reduce(gy, y, asel, mi, S, True, part)
    sums = part.view(S, nblk, 2, C).sum(1)
    xh = (a.float() - mi[:S * C].view(S, C)[seg][:, None, None, :]) * \
        mi[S * C:].view(S, C)[seg][:, None, None, :]
    for s_ in range(S):
        gs = g[seg == s_].reshape(-1, C)
        assert _rel(sums[s_, 0], gs.sum(0)) < 1e-3
        assert _rel(sums[s_, 1], (gs * xh[seg == s_].reshape(-1, C)).sum(0)) < 1e-3
