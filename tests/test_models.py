"""Model topology, parameter names, checkpoint contract and per-view BN semantics (CPU)."""
import pytest
import torch

from simclr_amd.models import (CentroidClassifier, ContrastiveModel, LinearClassifier,
                               NonLinearClassifier, SupervisedModel)
from simclr_amd.evaluation.probes import DownstreamDataset
from simclr_amd.utils.checkpoint import reference_state_dict, load_into, strip_prefix


@pytest.mark.parametrize("base,params,tensors,entries,conv1", [
    ("resnet18", 11_498_048, 65, 128, (64, 3, 3, 3)),
    ("resnet50", 27_970_624, 164, 326, (64, 3, 7, 7)),
])
def test_topology_matches_reference(base, params, tensors, entries, conv1):
    m = ContrastiveModel(base)
    assert sum(p.numel() for p in m.parameters()) == params
    assert len(list(m.parameters())) == tensors
    sd = reference_state_dict(m)
    assert len(sd) == entries
    assert all(k.startswith("module.") for k in sd)
    assert tuple(sd["module.f.conv1.weight"].shape) == conv1
    assert "module.g.projection_head.linear2.weight" in sd
    assert "module.g.projection_head.linear2.bias" not in sd
    assert "module.f.layer2.0.downsample.1.running_var" in sd
    assert all(v.dtype in (torch.float32, torch.int64) and v.is_contiguous() for v in sd.values())


def test_reference_stem_quirks():
    r18 = ContrastiveModel("resnet18").f
    assert r18.conv1.padding == (3, 3) and r18.conv1.kernel_size == (3, 3)
    x = torch.randn(2, 3, 32, 32)
    assert r18.conv1(x).shape[-1] == 36  # padding-3 stem gives 36x36 maps (Q6)
    r50 = ContrastiveModel("resnet50").f
    assert r50.conv1.kernel_size == (7, 7) and r50.conv1.stride == (2, 2)  # Q7
    c50 = ContrastiveModel("resnet50", cifar_stem=True).f
    assert c50.conv1.kernel_size == (3, 3) and c50.conv1.padding == (1, 1)


def test_segmented_bn_equals_two_forwards():
    """One forward of [v0; v1] with segments=2 == the reference's two forwards (train mode):
    same outputs and same running statistics."""
    torch.manual_seed(0)
    a = ContrastiveModel("resnet18")
    b = ContrastiveModel("resnet18")
    b.load_state_dict(a.state_dict())
    v0, v1 = torch.randn(4, 3, 32, 32), torch.randn(4, 3, 32, 32)
    z = a(torch.cat([v0, v1]), segments=2)
    z0, z1 = b(v0), b(v1)
    assert torch.allclose(z, torch.cat([z0, z1]), atol=1e-4, rtol=1e-4)
    sa, sb = a.state_dict(), b.state_dict()
    for k in sa:
        if "running" in k or "num_batches" in k:
            assert torch.allclose(sa[k].float(), sb[k].float(), atol=1e-5), k


def test_checkpoint_roundtrip(tmp_path):
    torch.manual_seed(1)
    m = ContrastiveModel("resnet18")
    p = tmp_path / "epoch=1-x.pt"
    torch.save(reference_state_dict(m), p)
    m2 = ContrastiveModel("resnet18")
    missing, unexpected = load_into(m2, p, strict=True)
    assert not missing and not unexpected
    for (k, v), (_, w) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(v, w), k
    sd = torch.load(p, weights_only=True)
    assert list(strip_prefix(sd)) == list(m.state_dict())


def test_classifiers():
    X = torch.tensor([[1.0, 0.0], [0.9, 0.1], [0.0, 1.0], [0.2, 0.8]])
    Y = torch.tensor([0, 0, 1, 1])
    w = CentroidClassifier.create_weights(DownstreamDataset(X, Y), 2)
    assert torch.allclose(w[:, 0], X[:2].mean(0)) and w.shape == (2, 2)
    assert CentroidClassifier(w)(X).argmax(1).tolist() == [0, 0, 1, 1]
    assert LinearClassifier(2, 3)(X).shape == (4, 3)
    nl = NonLinearClassifier(2, 3)
    assert nl(X).shape == (4, 3)
    assert {n for n, _ in nl.named_parameters()} >= {"classifier.linear1.weight",
                                                     "classifier.linear2.bias"}
    sm = SupervisedModel("resnet18", num_classes=10)
    assert sm(torch.randn(2, 3, 32, 32)).shape == (2, 10)
