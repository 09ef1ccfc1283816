"""HIP kernels of csrc/eval.hip against PyTorch fp32 references: max pool with argmax (SURVEY
K2), cross-entropy + top-k rank (K10), centroid class sums (K11); and the ImageNet-stem
ResNet-50 (reference model.py:90-92) running its max pool on the kernel."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ops():
    from simclr_amd.ops import _ext
    _ext.require()
    return _ext.ops()


@pytest.mark.parametrize("shape", [(8, 64, 16, 16), (4, 64, 15, 17), (2, 128, 112, 112)])
def test_maxpool_fwd_bwd_match_torch(shape):
    from simclr_amd.ops.pooling import MaxPool2d
    _ops()
    torch.manual_seed(0)
    x = torch.randn(*shape, device=DEV).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last).requires_grad_(True)
    y = MaxPool2d(3, 2, 1)(x)
    xr = x.detach().float().requires_grad_(True)
    yr = F.max_pool2d(xr, 3, 2, 1)
    assert y.shape == yr.shape
    assert torch.equal(y.float(), yr)  # max of bf16 values is exact
    g = torch.randn_like(yr).to(torch.bfloat16)
    y.backward(g)
    yr.backward(g.float())
    # each input gathers <= 4 window gradients: bf16 rounding of that sum only
    assert torch.allclose(x.grad.float(), xr.grad, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("B,C", [(512, 10), (300, 100), (64, 1000)])
def test_ce_topk_matches_torch(B, C):
    from simclr_amd.ops.classify import ce_rank, cross_entropy
    _ops()
    torch.manual_seed(1)
    z = torch.randn(B, C, device=DEV) * 3
    y = torch.randint(0, C, (B,), device=DEV)
    loss, rank = ce_rank(z, y)
    ref = F.cross_entropy(z, y, reduction="none")
    assert torch.allclose(loss, ref, rtol=1e-5, atol=1e-5)
    for k in (1, 5):
        kk = min(k, C)
        top = torch.topk(z, kk, dim=1)[1]
        assert int((rank < kk).sum()) == int((top == y[:, None]).any(1).sum())
    zr = z.clone().requires_grad_(True)
    zh = z.clone().requires_grad_(True)
    F.cross_entropy(zr, y).backward()
    lh = cross_entropy(zh, y)
    lh.backward()
    assert abs(float(lh) - float(F.cross_entropy(z, y))) < 1e-5
    assert torch.allclose(zh.grad, zr.grad, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("N,D,NC", [(5000, 512, 10), (50000, 2048, 10), (1000, 128, 100)])
def test_class_means_match_index_add(N, D, NC):
    from simclr_amd.ops.classify import class_means
    _ops()
    torch.manual_seed(2)
    X = torch.randn(N, D, device=DEV)
    y = torch.randint(0, NC, (N,), device=DEV)
    got = class_means(X, y, NC)
    s = torch.zeros(NC, D, dtype=torch.float64, device=DEV).index_add_(0, y, X.double())
    ref = (s / torch.bincount(y, minlength=NC).double()[:, None]).float()
    assert torch.allclose(got, ref, rtol=1e-4, atol=1e-5)


def test_imagenet_stem_resnet50_uses_hip_maxpool():
    """The reference's resnet50 (7x7/s2 stem + max pool on 32x32) through the HIP path."""
    from simclr_amd.models.contrastive import ContrastiveModel
    from simclr_amd.ops import pooling_hip
    _ops()
    calls = []
    orig = pooling_hip.MaxPoolHipFn.forward

    def spy(ctx, *a):
        calls.append(1)
        return orig(ctx, *a)
    pooling_hip.MaxPoolHipFn.forward = staticmethod(spy)
    try:
        torch.manual_seed(0)
        m = ContrastiveModel(base_cnn="resnet50", d=128, cifar_stem=None).to(DEV)
        from simclr_amd.parallel.flat import FlatParamStore
        store = FlatParamStore(m, torch.device(DEV, 0), shadow_dtype=torch.bfloat16)
        m.train()
        x = torch.rand(64, 8, 32, 32, device=DEV).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        z = m(x, segments=2)
        z.float().pow(2).sum().backward()
        store.finish()
        torch.cuda.synchronize()
        assert calls, "HIP max pool did not run"
        assert bool(torch.isfinite(store.grad).all())
    finally:
        pooling_hip.MaxPoolHipFn.forward = staticmethod(orig)


def _topk_correct(z, y, k):
    return (torch.topk(z, k, dim=1)[1] == y[:, None]).any(1)


def test_ce_topk_nan_logits_follow_torch_topk():
    """A diverged probe (NaN logits) must not read as 100 % accurate: a NaN target logit is
    never correct and a NaN of another class ranks above the target (torch.topk's order)."""
    from simclr_amd.ops.classify import ce_rank
    _ops()
    torch.manual_seed(3)
    B, C = 256, 10
    z = torch.randn(B, C, device=DEV)
    y = torch.randint(0, C, (B,), device=DEV)
    z[:64] = float("nan")                                  # whole rows NaN
    z[64:128, 3] = float("nan")                            # one NaN class per row
    z[128:160].scatter_(1, y[128:160, None], float("nan"))  # NaN target logit only
    _, rank = ce_rank(z, y)
    nan_t = torch.isnan(z.gather(1, y[:, None])).view(-1)
    assert bool((rank[nan_t] == C).all())  # topk may pick a NaN target: we never count it
    for k in (1, 5):
        assert torch.equal((rank < k)[~nan_t], _topk_correct(z, y, k)[~nan_t]), k
