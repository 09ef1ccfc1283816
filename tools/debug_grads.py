"""Debug helper: how far are the bf16 HIP-path gradients from an fp32 torch-path gradient of the
same network/input, and are they deterministic?  Loss = Σ h·w (backbone features)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(mode, x, w, base="resnet50", stem=True, perm=None):
    from simclr_amd.models.contrastive import ContrastiveModel
    from simclr_amd.parallel import state as pstate
    from simclr_amd.parallel.flat import FlatParamStore
    pstate.reset()
    dev = torch.device("cuda", 0)
    pstate.get().device = dev
    torch.manual_seed(0)
    m = ContrastiveModel(base_cnn=base, d=128, cifar_stem=stem).to(dev)
    m.f.use_fused_stages = mode == "fused"
    damp = float(os.environ.get("DAMP", "1.0"))
    if damp != 1.0:  # damped residual branches: a well-conditioned (near-identity) network
        with torch.no_grad():
            for layer in (m.f.layer1, m.f.layer2, m.f.layer3, m.f.layer4):
                for blk in layer:
                    last = blk.bn3 if hasattr(blk, "bn3") else blk.bn2
                    last.weight.mul_(damp)
    store = FlatParamStore(m, dev, shadow_dtype=torch.bfloat16)
    m.train()
    if mode == "fp32":
        with torch.no_grad():
            store.master.copy_(store.shadow.float())
        store.shadow = None
        for sl in store.slots:
            sl.shadow = None
        xin = x.float()[:, :3].contiguous()
    else:
        xin = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    h = m.encode(xin, segments=2)
    loss = (h.float() * w).sum()
    store.zero_grad()
    loss.backward()
    torch.cuda.synchronize()
    return h.detach().float(), store.grad.clone(), store


def main():
    base = sys.argv[1] if len(sys.argv) > 1 else "resnet50"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    stem = None if base == "resnet18" else True
    g = torch.Generator().manual_seed(1)
    x = torch.rand(2 * n, 8, 32, 32, generator=g).cuda()
    x = x.to(torch.bfloat16).float()
    F = 512 if base == "resnet18" else 2048
    w = torch.randn(2 * n, F, generator=g).cuda()
    h32, g32, store = run("fp32", x, w, base, stem)
    hm, gm, _ = run("module", x, w, base, stem)
    hf, gf, _ = run("fused", x, w, base, stem)
    hf2, gf2, _ = run("fused", x, w, base, stem)

    def rel(a, b):
        return float((a - b).norm() / (b.norm() + 1e-12))

    print(f"h: module-vs-fp32 {rel(hm, h32):.4f} fused-vs-fp32 {rel(hf, h32):.4f} "
          f"fused-rerun {rel(hf2, hf):.2e}")
    print(f"grad: module-vs-fp32 {rel(gm, g32):.4f} fused-vs-fp32 {rel(gf, g32):.4f} "
          f"fused-rerun {rel(gf2, gf):.2e} module-vs-fused {rel(gm, gf):.4f}")
    for (o, k), name in list(zip(store.segments(), store.names)):
        if not name.startswith("f."):
            continue
        r = g32[o:o + k]
        if r.norm() < 1e-12:
            continue
        print(f"  {name:45s} |g|={float(r.norm()):.3e} mod={rel(gm[o:o+k], r):.3f} "
              f"fus={rel(gf[o:o+k], r):.3f} rerun={rel(gf2[o:o+k], gf[o:o+k]):.1e}")


if __name__ == "__main__":
    main()
