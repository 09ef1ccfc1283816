"""Three-way comparison of the fused stage executor (models/fused.py) against the per-module bf16
path and an fp32 torch run of the same weights, on a WELL-CONDITIONED network.

Why conditioned: at random init a bf16 ResNet-50 is chaotic — the per-stage error of BOTH bf16
paths against fp32 grows ~3x per stage (1.3 % at layer1 → 39 % at layer4, GPUTEST_r04), and the
NT-Xent loss of nearly identical embeddings turns that into gradients that move by tens of
percent.  A comparison at that noise floor cannot see a few-percent kernel defect.  Here

  * every residual block's last BatchNorm starts at γ = ``gamma_last`` (the "zero-init residual"
    recipe with a non-zero value, so every weight still gets a gradient): each block is close to
    the identity, rounding errors no longer amplify from stage to stage (measured: 0.6 % at
    layer1 → 2.6 % at layer4 on both bf16 paths);
  * every other BatchNorm starts at γ = 0.25, β = 1, so a ReLU input sits ~4 σ above zero: at
    init the ReLU masks are what makes the gradient chaotic — a 1-2 % rounding difference flips
    the masks of the units near zero, and a flipped unit passes its whole gradient or none, so
    with the default init BOTH bf16 paths' parameter gradients were 30 % (ResNet-50) / 15 %
    (ResNet-18) from fp32 for EVERY parameter (measured) even though the forward agreed to 2 %.
    The mask logic itself (mode 3 / 4 epilogues, block-output bitmask) has per-kernel tests;
  * the backward is driven by a fixed random projection of the backbone features h (the fused
    executor's output after the average pool), L = Σ h·R / N, instead of NT-Xent on the
    projection head's z: at init the features of different images are nearly equal, so the
    head's BatchNorm1d (x − mean) / std amplifies the bf16 rounding of h into a ~25 % error of z
    and of every gradient (measured), and the NT-Xent gradient is itself a small difference of
    nearly equal rows.  The head and the NT-Xent kernels have their own fp32 tests.

Both paths then sit at the ~1 % bf16 floor at every stage and for every parameter gradient, and
a 2 % error in one conv (``mutate``) stands out.  Reference semantics: torchvision
Bottleneck / BasicBlock with SyncBN (``/root/reference/model.py:76-114``, main.py:112-116,176).
"""
from __future__ import annotations

import torch

DEV = "cuda"
STAGES = ("layer1", "layer2", "layer3", "layer4")


def _bf(t):
    return t.to(torch.bfloat16)


def _model(base, stem, device, gamma_last, gamma=0.25, beta=1.0):
    from simclr_amd.models.contrastive import ContrastiveModel
    from simclr_amd.models.resnet import BasicBlock, Bottleneck
    from simclr_amd.ops.batchnorm import _BatchNormBase
    from simclr_amd.parallel import state as pstate
    from simclr_amd.parallel.flat import FlatParamStore
    pstate.reset()
    pstate.get().device = device
    torch.manual_seed(0)
    m = ContrastiveModel(base_cnn=base, d=128, cifar_stem=stem).to(device)
    if gamma_last is not None:
        with torch.no_grad():
            for mod in m.f.modules():
                if isinstance(mod, _BatchNormBase):
                    mod.weight.fill_(gamma)
                    mod.bias.fill_(beta)
            for mod in m.f.modules():
                if isinstance(mod, Bottleneck):
                    mod.bn3.weight.fill_(gamma_last)
                elif isinstance(mod, BasicBlock):
                    mod.bn2.weight.fill_(gamma_last)
    store = FlatParamStore(m, device, shadow_dtype=torch.bfloat16)
    m.train()
    return m, store


def run_three(base, stem, batch, monkeypatch, block_out=True, gamma_last=0.2, mutate=None,
              loss="projection"):
    """Run the module, fused and fp32 paths from identical weights / input.  ``mutate``:
    ``("fwd" | "dgrad", block name, conv index)`` scales that conv's forward output (after its
    BatchNorm statistics were taken, i.e. what the consumers read is 2 % off) or its input
    gradient by 1.02 inside the fused executor.  Returns a metrics dict."""
    from simclr_amd.loss.ntxent import NTXent
    from simclr_amd.models.fused import FusedStages
    monkeypatch.setattr(FusedStages, "BLOCK_OUT_PROLOGUE", bool(block_out))
    dev = torch.device(DEV, 0)
    torch.manual_seed(5)
    x = _bf(torch.rand(2 * batch, 8, 32, 32, device=dev)).contiguous(
        memory_format=torch.channels_last)
    stages = {}
    orig_fwd = FusedStages.forward

    def rec_fwd(self, xn):  # the fused executor's block outputs, per stage (last block wins)
        out, tapes = orig_fwd(self, xn)
        for b, tp in zip(self.blocks, tapes):
            stages["fused"][b.name.split(".")[0]] = tp.out.float().permute(0, 3, 1, 2).clone()
        return out, tapes
    monkeypatch.setattr(FusedStages, "forward", rec_fwd)
    bstages = {}  # mode -> {stage: gradient w.r.t. the stage's input (fp32, NCHW)}
    orig_bb = FusedStages._block_backward

    def rec_bb(self, ops, st, S, b, tp, g, pre, prev):
        dx, h = orig_bb(self, ops, st, S, b, tp, g, pre, prev)
        if b.name.endswith(".0"):  # the input of a stage's first block
            bstages["fused"][b.name.split(".")[0]] = dx.float().permute(0, 3, 1, 2).clone()
        return dx, h
    monkeypatch.setattr(FusedStages, "_block_backward", rec_bb)
    if mutate is not None:
        kind, bname, ci = mutate
        if kind == "fwd":
            orig_conv = FusedStages._conv_fwd

            def conv_fwd(self, ops, xn, cs, *a, **kw):
                a_, partial, nblk = orig_conv(self, ops, xn, cs, *a, **kw)
                b = next(b for b in self.blocks if b.name == bname)
                if cs is b.convs[ci]:
                    a_.mul_(1.02)  # after the epilogue's statistics partials
                return a_, partial, nblk
            monkeypatch.setattr(FusedStages, "_conv_fwd", conv_fwd)
        else:
            orig_dgrad = FusedStages._dgrad

            def dgrad(self, ops, dyn, cs, *a, **kw):
                dx, part, nb = orig_dgrad(self, ops, dyn, cs, *a, **kw)
                b = next(b for b in self.blocks if b.name == bname)
                if cs is b.convs[ci]:
                    dx.mul_(1.02)
                return dx, part, nb
            monkeypatch.setattr(FusedStages, "_dgrad", dgrad)
    res = {}
    torch.manual_seed(6)
    proj = None
    for mode in ("module", "fused", "fp32"):
        m2, store2 = _model(base, stem, dev, gamma_last)
        m2.f.use_fused_stages = mode == "fused"
        stages[mode] = {}
        bstages[mode] = {}
        hooks = []
        if mode != "fused":
            for ln in STAGES:
                hooks.append(getattr(m2.f, ln)[-1].register_forward_hook(
                    lambda mod, inp, out, ln=ln, mode=mode:
                    stages[mode].__setitem__(ln, out.detach().float().clone())))

                def pre(mod, inp, ln=ln, mode=mode):
                    if inp[0].requires_grad:
                        inp[0].register_hook(lambda g, ln=ln, mode=mode: bstages[mode].__setitem__(
                            ln, g.detach().float().clone()))
                hooks.append(getattr(m2.f, ln)[0].register_forward_pre_hook(pre))
        if mode == "fp32":
            with torch.no_grad():  # same (bf16-representable) weights, fp32 compute
                store2.master.copy_(store2.shadow.float())
            store2.shadow = None
            for sl in store2.slots:
                sl.shadow = None
        store2.zero_grad()
        xin = x.float()[:, :3].contiguous() if mode == "fp32" else x
        if loss in ("projection", "energy"):  # the backbone alone (the executor's output)
            z = m2.encode(xin, segments=2)
        else:
            z = m2(xin, segments=2)
        if proj is None:
            proj = torch.randn(z.shape, device=dev, dtype=torch.float32)
        if loss == "projection":
            lval = (z.float() * proj).sum() / z.shape[0]
        elif loss == "energy":
            lval = 0.5 * (z.float() * (z.float() + proj)).sum() / z.shape[0]
        else:
            lval = NTXent(temperature=0.5)(z)
        lval.backward()
        torch.cuda.synchronize()
        if mode == "fused":
            ex = m2.f.__dict__.get("_fused_cache", {}).get(2)
            assert ex is not None and ex.calls == 1, "fused executor did not run"
            res["launch_counts"] = (len(ex.blocks), ex.dual_launches, ex.out_apply_calls)
        for h in hooks:
            h.remove()
        res[mode] = (float(lval.detach()), store2.grad.clone(),
                     [(n, b.float().clone()) for n, b in m2.named_buffers() if "running" in n])
    _, store = _model(base, stem, dev, gamma_last)
    gm, gf, gr = res["module"][1], res["fused"][1], res["fp32"][1]

    def rel(u, w):
        return (u - w).norm().item() / (w.norm().item() + 1e-12)

    out = {"stage": {}, "param": {}, "buffers": {}, "launch_counts": res["launch_counts"],
           "loss": (res["fused"][0], res["module"][0], res["fp32"][0])}
    out["stage_fm"], out["param_fm"], out["bstage"] = {}, {}, {}
    for ln in STAGES:
        w = bstages["fp32"].get(ln)
        if w is not None and ln in bstages["fused"] and ln in bstages["module"]:
            out["bstage"][ln] = (rel(bstages["fused"][ln], w), rel(bstages["module"][ln], w))
            out["bstage_fm"] = out.get("bstage_fm", {})
            out["bstage_fm"][ln] = rel(bstages["fused"][ln], bstages["module"][ln])
    for ln in STAGES:
        w = stages["fp32"][ln]
        out["stage"][ln] = (rel(stages["fused"][ln], w), rel(stages["module"][ln], w))
        out["stage_fm"][ln] = rel(stages["fused"][ln], stages["module"][ln])
    norms = sorted(gr[o:o + n_].norm().item() for o, n_ in store.segments())
    med = norms[len(norms) // 2]
    out["param_small"] = set()
    for (o, n_), name in zip(store.segments(), store.names):
        w = gr[o:o + n_]
        if w.norm().item() < 1e-8:
            continue
        if w.norm().item() < 1e-3 * med:  # an fp32 gradient that is itself round-off
            out["param_small"].add(name)
        out["param"][name] = (rel(gf[o:o + n_], w), rel(gm[o:o + n_], w))
        out["param_fm"][name] = rel(gf[o:o + n_], gm[o:o + n_])
    out["total_grad"] = (rel(gf, gr), rel(gm, gr))
    for (name, u), (_, v), (_, w) in zip(res["fused"][2], res["module"][2], res["fp32"][2]):
        out["buffers"][name] = (rel(u, w), rel(v, w))
    return out


# Bounds on the conditioned network, calibrated on MI355X (ResNet-50 CIFAR stem, batch 32 x 2
# views; tools/fused_calib.py).  Forward stage outputs: 0.30 / 0.41 / 0.44 / 0.65 % from fp32 on
# BOTH bf16 paths (fused / module within 2 % of each other); input gradients of the stages
# 1.50 / 1.35 / 1.18 / 0.89 % on both (ratio 1.000-1.004); running statistics <= 0.09 %.  The
# norms of these error tensors concentrate (millions of independent rounding errors), so the
# fused path's error tracks the module path's to a fraction of a percent, and a defect that
# adds a coherent component shows as a ratio: a 2 % error in one layer3 conv moved them by
# +15 % (its input gradient) to +35 % (its forward output), and the running statistics of the
# next BatchNorm 100x.  Per-parameter gradients are only checked grossly: each is a sum of
# ~1e5 products whose rounding noise does not average out (7-10 % from fp32 for a conv weight
# on both paths, 10-15 % apart from each other), and the biases of BatchNorms that feed a
# BatchNorm through 1x1 convs have an fp32 gradient that is itself round-off (some BatchNorm
# biases measured at 2.2x the module path's error: the gross bound is 3x + 0.1).
STAGE_ABS, STAGE_RATIO, STAGE_SLACK = 0.02, 1.10, 0.001
BSTAGE_ABS, BSTAGE_RATIO, BSTAGE_SLACK = 0.045, 1.06, 0.0005
BUFFER_RATIO, BUFFER_SLACK = 1.5, 0.002
TOTAL_RATIO, TOTAL_SLACK = 1.25, 0.01
PARAM_RATIO, PARAM_SLACK = 3.0, 0.1


def violations(mt):
    """Every bound the fused path breaks (empty list = pass)."""
    bad = []
    for ln, (ef, em) in mt["stage"].items():
        if ef > STAGE_ABS or ef > STAGE_RATIO * em + STAGE_SLACK:
            bad.append(("stage", ln, ef, em))
    for ln, (ef, em) in mt["bstage"].items():
        if ef > BSTAGE_ABS or ef > BSTAGE_RATIO * em + BSTAGE_SLACK:
            bad.append(("input-grad", ln, ef, em))
    for name, (ef, em) in mt["buffers"].items():
        if ef > BUFFER_RATIO * em + BUFFER_SLACK:
            bad.append(("buffer", name, ef, em))
    ef, em = mt["total_grad"]
    if ef > TOTAL_RATIO * em + TOTAL_SLACK:
        bad.append(("grad", "total", ef, em))
    for name, (ef, em) in mt["param"].items():
        if name in mt["param_small"]:
            continue
        if ef > PARAM_RATIO * em + PARAM_SLACK:
            bad.append(("grad", name, ef, em))
    return bad


def _dist(vals):
    v = sorted(vals)
    if not v:
        return None
    return tuple(round(v[int(q * (len(v) - 1))], 5) for q in (0.5, 0.9, 1.0))


def summary(mt, top=6):
    worst = sorted(mt["param"].items(), key=lambda kv: -kv[1][0])[:top]
    ratio = sorted(((k, a / max(b, 1e-9), a, b) for k, (a, b) in mt["param"].items()),
                   key=lambda t: -t[1])[:top]
    convs = [kv for kv in mt["param"].items() if "conv" in kv[0] or "downsample.0" in kv[0]]
    bns = [kv for kv in mt["param"].items() if kv not in convs]
    fm = sorted(mt["param_fm"].items(), key=lambda kv: -kv[1])
    fmc = [v for k, v in fm if "conv" in k or "downsample.0" in k]
    return {"stage": {k: (round(a, 5), round(b, 5)) for k, (a, b) in mt["stage"].items()},
            "stage_fm": {k: round(v, 5) for k, v in mt["stage_fm"].items()},
            "bstage": {k: (round(a, 5), round(b, 5)) for k, (a, b) in mt["bstage"].items()},
            "bstage_fm": {k: round(v, 5) for k, v in mt.get("bstage_fm", {}).items()},
            "fm_conv_q50_q90_max": _dist(fmc),
            "fm_worst": [(k, round(v, 5)) for k, v in fm[:top]],
            "conv_grad_q50_q90_max": (_dist([a for _, (a, b) in convs]),
                                      _dist([b for _, (a, b) in convs])),
            "bn_grad_q50_q90_max": (_dist([a for _, (a, b) in bns]),
                                    _dist([b for _, (a, b) in bns])),
            "worst_ratio": [(k, round(r, 3), round(a, 5), round(b, 5)) for k, r, a, b in ratio],
            "worst_grads": [(k, round(a, 5), round(b, 5)) for k, (a, b) in worst],
            "total_grad": tuple(round(v, 5) for v in mt["total_grad"]),
            "worst_buffer": max(((k, round(a, 5), round(b, 5))
                                 for k, (a, b) in mt["buffers"].items()), key=lambda t: t[1]),
            "loss": tuple(round(v, 5) for v in mt["loss"])}
