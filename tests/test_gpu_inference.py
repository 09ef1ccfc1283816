"""Inference (eval-mode) parity of the HIP path: every probe, feature export and supervised
validation runs the model in eval mode (/root/reference/eval.py:31-58,
save_features.py:20-77, supervised.py:30-58) — BatchNorm from running statistics
(``bn_apply_eval``), convolutions without statistics epilogues, the max pool of the ImageNet
stem and the head's BatchNorm1d in eval.  The bf16 HIP model is compared with the fp32 torch
model holding identical weights and non-trivial running statistics, on un-augmented inputs from
the production EvalLoader."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _randomise_bn(model, seed):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for m in model.modules():
            if hasattr(m, "running_mean") and m.running_mean is not None:
                C = m.running_mean.numel()
                m.running_mean.copy_((torch.rand(C, generator=g) - 0.5) * 0.4)
                m.running_var.copy_(0.5 + 1.5 * torch.rand(C, generator=g))
                m.weight.copy_(0.5 + torch.rand(C, generator=g))
                m.bias.copy_((torch.rand(C, generator=g) - 0.5) * 0.4)


def _pair(kind, base, stem, seed=0):
    from simclr_amd.models.contrastive import ContrastiveModel, SupervisedModel
    from simclr_amd.parallel.flat import FlatParamStore

    def make():
        torch.manual_seed(seed)
        if kind == "contrastive":
            return ContrastiveModel(base_cnn=base, d=128, cifar_stem=stem)
        return SupervisedModel(base_cnn=base, num_classes=10, cifar_stem=stem)
    hip = make().to(DEV)
    _randomise_bn(hip, seed + 1)
    ref = make().to(DEV)
    ref.load_state_dict(hip.state_dict())
    store = FlatParamStore(hip, DEV, shadow_dtype=torch.bfloat16)
    store.refresh_shadow()
    hip.eval()
    ref.eval()
    return hip, ref, store


def _inputs(n=128):
    from simclr_amd.data.datasets import synthetic_dataset
    from simclr_amd.data.loader import EvalLoader
    x, _ = next(iter(EvalLoader(synthetic_dataset(n, 10, seed=3), n, DEV)))
    return x


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def _ref_forward(fn, x):
    from simclr_amd.ops import registry
    old = registry.get_backend()
    registry.set_backend("torch")
    try:
        return fn(x.float()[:, :3].contiguous())
    finally:
        registry.set_backend(old)


@pytest.mark.parametrize("base,stem", [("resnet18", None), ("resnet50", None), ("resnet50", True)],
                         ids=["r18-refstem", "r50-imagenet-stem", "r50-cifar-stem"])
def test_eval_mode_encode_and_forward_match_fp32(base, stem):
    from simclr_amd.ops import _ext
    _ext.require()
    hip, ref, _ = _pair("contrastive", base, stem)
    x = _inputs()
    with torch.no_grad():
        h, z = hip.encode(x), hip(x)
        hr = _ref_forward(ref.encode, x)
        zr = _ref_forward(ref.forward, x)
    assert h.shape == hr.shape and z.shape == zr.shape
    eh, ez = _rel(h, hr), _rel(z, zr)
    print(f"{base} stem={stem}: rel(h)={eh:.2e} rel(z)={ez:.2e}")
    assert eh <= 2e-2 and ez <= 2e-2, (eh, ez)
    # eval mode leaves the running statistics untouched
    for (n1, b1), (n2, b2) in zip(hip.named_buffers(), ref.named_buffers()):
        assert torch.equal(b1.float(), b2.float()), n1


@pytest.mark.parametrize("base,stem", [("resnet18", None), ("resnet50", True)])
def test_supervised_validation_logits_match_fp32(base, stem):
    from simclr_amd.ops import _ext
    from simclr_amd.ops.classify import ce_rank
    _ext.require()
    hip, ref, _ = _pair("supervised", base, stem, seed=5)
    x = _inputs()
    y = torch.randint(0, 10, (x.shape[0],), device=DEV)
    with torch.no_grad():
        out = hip(x).float()
        outr = _ref_forward(ref.forward, x).float()
    e = _rel(out, outr)
    print(f"supervised {base}: rel(logits)={e:.2e}")
    assert e <= 2e-2, e
    # the validation counts (supervised.py validation(): CE sum, rank-0 = correct)
    l, r = ce_rank(out, y)
    lr = torch.nn.functional.cross_entropy(outr, y, reduction="sum")
    assert abs(float(l.sum()) - float(lr)) <= 2e-2 * abs(float(lr))
