"""The ImageNet stem's space-to-depth form (models/fused.py ``stem_s2d``; csrc/eval.hip
k_stem_s2d): a 7x7 / stride-2 / pad-3 conv over 3 channels equals a 4x4 / stride-1 / unpadded
conv over the 2x2 space-to-depth of the padded image with the folded kernel, and the folded
kernel's weight gradient unfolds to the 7x7 one.  fp64 on the CPU: the identity is exact up to
summation order.  Reference stem: /root/reference/model.py (torchvision resnet50 conv1)."""
import pytest
import torch
import torch.nn.functional as F

from simclr_amd.models.fused import FusedStages


def s2d_reference(img_nhwc: torch.Tensor, creal: int, P: int = 3) -> torch.Tensor:
    """[N, H, W, C] -> [N, (H+2P)/2, (W+2P)/2, 16], channel (dy * 2 + dx) * 4 + c."""
    x = img_nhwc[..., :4].clone()
    x[..., creal:] = 0
    x = F.pad(x, (0, 0, P, P, P, P))
    N, Hp, Wp, _ = x.shape
    return x.view(N, Hp // 2, 2, Wp // 2, 2, 4).permute(0, 1, 3, 2, 4, 5).reshape(
        N, Hp // 2, Wp // 2, 16)


@pytest.mark.parametrize("H", [32, 30, 14])
def test_s2d_conv_and_weight_gradient_identity(H):
    torch.manual_seed(3)
    N, Co = 2, 8
    img = torch.randn(N, H, H, 8, dtype=torch.float64)
    w = torch.randn(Co, 3, 7, 7, dtype=torch.float64)
    ref = F.conv2d(img[..., :3].permute(0, 3, 1, 2), w, None, 2, 3)
    xs = s2d_reference(img, 3)
    # fold as the executor does (its shadow cast is bf16: fold an fp64 copy the same way)
    w8 = F.pad(w.permute(0, 2, 3, 1), (0, 1, 0, 1, 0, 1))
    ws = w8.view(Co, 4, 2, 4, 2, 4).permute(0, 1, 3, 2, 4, 5).reshape(Co, 4, 4, 16)
    out = F.conv2d(xs.permute(0, 3, 1, 2), ws.permute(0, 3, 1, 2), None, 1, 0)
    assert out.shape == ref.shape
    assert torch.allclose(out, ref, rtol=1e-10, atol=1e-10)
    # the executor's bf16 fold is this fold, cast
    fold = FusedStages._s2d_weight(w.float())
    assert torch.equal(fold.float(), ws.to(torch.bfloat16).float())
    # weight gradient: dW of the 4x4 form, unfolded, equals dW of the 7x7 form
    dy = torch.randn_like(ref)
    gref = torch.nn.grad.conv2d_weight(img[..., :3].permute(0, 3, 1, 2), w.shape, dy, 2, 3)
    gs = torch.nn.grad.conv2d_weight(xs.permute(0, 3, 1, 2), (Co, 16, 4, 4), dy, 1, 0)
    out_g = torch.empty(Co, 7, 7, 3, dtype=torch.float64)
    FusedStages._s2d_unfold_grad(gs.permute(0, 2, 3, 1).contiguous(), out_g)
    assert torch.allclose(out_g.permute(0, 3, 1, 2), gref, rtol=1e-10, atol=1e-10)
