"""Teacher-forced per-op check of the production fused executor at batch 512 (VERDICT r5 item 3;
harness: tests/_teacher_forced.py).  Every conv's forward output, input gradient and weight
gradient, every BatchNorm's statistics, dγ / dβ and input-gradient coefficients, every block
output and ReLU mask of one real training step is compared against fp32 torch on the same bf16
operands — the autotuned production tiles and the side-stream tile cap included.  A 2 % defect
in one layer3 conv's weight gradient must be caught; without it every bound holds.
Reference: /root/reference/model.py:76-114, main.py:112-116."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _report(tag, errors):
    from _teacher_forced import summary
    for kind, (n, worst, name) in sorted(summary(errors).items()):
        print(f"{tag} {kind:6s} n={n:3d} max={worst:.2e} ({name})")


@pytest.mark.timeout(600)
@pytest.mark.parametrize("base,stem", [("resnet50", True), ("resnet18", None), ("resnet50", None)])
def test_teacher_forced_every_op_batch512(base, stem, monkeypatch):
    """(resnet50, None) is the reference's ResNet-50 (ImageNet 7x7/s2 stem + max-pool on 32x32):
    its stem runs as the fused BN + ReLU + max-pool forward and max-pool / ReLU / BN backward."""
    from _teacher_forced import BOUNDS, run_step, violations
    errors, counts, rec = run_step(base, stem, 512, monkeypatch)
    _report(base, errors)
    bad = violations(errors)
    assert not bad, bad[:10]
    # coverage: every conv of the backbone (stem included) checked forward, dgrad and weight
    # gradient; every BatchNorm's statistics and backward
    nconv = sum(len(b.convs) + (b.down is not None) for b in rec.blocks) + 1
    assert counts["y"] == nconv, counts
    assert counts["dW"] == nconv, counts
    assert counts["dx"] >= nconv - 1, counts  # the stem needs no input gradient
    assert counts["bnfwd"] == 2 * nconv, counts
    assert counts["dgb"] == 2 * nconv, counts
    assert counts["bnbwd"] >= nconv - 1, counts
    pooled = rec.stem_tape is not None and rec.stem_tape.pool is not None
    assert pooled == (stem is None and base == "resnet50"), "pooled stem not fused"
    assert counts["out"] == len(rec.blocks) + 1, counts
    assert counts["mask"] == counts["out"], counts
    if base == "resnet50":
        assert nconv == 53


@pytest.mark.timeout(600)
@pytest.mark.parametrize("factor", [1.02, 1.002])
def test_teacher_forced_catches_weight_gradient_defect(factor, monkeypatch):
    """One layer3 conv's weight gradient scaled inside the executor (on the stream that computed
    it): the per-op check must flag exactly that conv's dW."""
    from _teacher_forced import run_step, violations
    errors, _, _ = run_step("resnet50", True, 512, monkeypatch,
                            mutate_dw=("layer3.1.conv2", factor))
    bad = violations(errors)
    print(f"MUTATION dW layer3.1.conv2 x{factor}:", bad)
    assert [(k, n) for k, n, _ in bad] == [("dW", "layer3.1.conv2")], bad
