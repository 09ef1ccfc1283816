"""Per-layer microbenchmark of the implicit-GEMM conv kernels on the ResNet-50 CIFAR shapes.

For every distinct conv of the network (batch = 2 views x 512) it times forward, dgrad and wgrad
for every tile variant and prints achieved TFLOP/s and effective HBM GB/s (compulsory bytes).
Usage (GPU box): python tools/conv_bench.py [--batch 1024] [--model resnet50] [--imagenet-stem]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def conv_shapes(model: str, cifar_stem: bool, batch: int, size: int = 32):
    from simclr_amd.models import ContrastiveModel
    m = ContrastiveModel(model, cifar_stem=cifar_stem if cifar_stem else None)
    shapes = []
    hooks = []
    from simclr_amd.ops.conv import Conv2d

    def hook(mod, inp, out):
        x = inp[0]
        shapes.append((batch, x.shape[1], x.shape[2], x.shape[3], mod.out_channels,
                       mod.kernel_size[0], mod.stride[0], mod.padding[0]))
    for mod in m.modules():
        if isinstance(mod, Conv2d):
            hooks.append(mod.register_forward_hook(hook))
    with torch.no_grad():
        m.eval()
        m(torch.zeros(2, 3, size, size))
    uniq = []
    for s in shapes:
        if s not in uniq:
            uniq.append(s)
    return shapes, uniq


def timeit(fn, reps=10):
    fn()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--imagenet-stem", action="store_true")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from simclr_amd.ops import _ext
    from simclr_amd.ops.conv_hip import fwd_geom, conv_dgrad
    ops = _ext.ops()
    dev = torch.device("cuda", 0)
    allshapes, uniq = conv_shapes(a.model, not a.imagenet_stem, a.batch)
    counts = {s: allshapes.count(s) for s in uniq}
    rows = []
    tot_best = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    for (N, C, H, W, Co, k, s, p) in uniq:
        Cg = max(8, C)
        OH = (H + 2 * p - k) // s + 1
        OW = (W + 2 * p - k) // s + 1
        M = N * OH * OW
        flop = 2.0 * M * Co * k * k * C
        x = torch.randn(N, OH * 0 + H, W, Cg, device=dev).to(torch.bfloat16)
        w = (torch.randn(Co, k, k, Cg, device=dev) * 0.05).to(torch.bfloat16)
        y = torch.empty(N, OH, OW, Co, device=dev, dtype=torch.bfloat16)
        g = fwd_geom(N, H, W, Cg, OH, OW, k, k, s, p, Co)
        fw = {}
        for v in range(ops.igemm_nvariants()):
            if not ops.igemm_variant_ok(v, g, False, False):
                continue
            fw[v] = timeit(lambda: ops.igemm(x, w, y, None, None, g, None, None, 0, False, 0, None,
                                             None, v))
        dg = None
        if C >= 8 and C % 8 == 0 and C == Cg:
            dyn = torch.randn(N, OH, OW, Co, device=dev).to(torch.bfloat16)
            dg = timeit(lambda: conv_dgrad(ops, dyn, w, N, H, W, C, OH, OW, k, k, s, p, Co))
        wg = {}
        dyn = torch.randn(N, OH, OW, Co, device=dev).to(torch.bfloat16)
        out = torch.empty(Co, k, k, Cg, device=dev)
        for v in range(ops.wgrad_nvariants()):
            if not ops.wgrad_variant_ok(v, g, False, False):
                continue
            sp = ops.wgrad_splits(g, v)
            part = torch.empty(sp * Co * k * k * Cg, device=dev)
            wg[v] = timeit(lambda: ops.wgrad(dyn, x, part, out, g, sp, Cg, 0.0, None, None, 0,
                                             False, 1, v))
        bytes_f = 2.0 * (N * H * W * Cg + M * Co)
        bf = min(fw.values())
        bw = min(wg.values())
        n = counts[(N, C, H, W, Co, k, s, p)]
        tot_best["fwd"] += bf * n
        tot_best["wgrad"] += bw * n
        if dg:
            tot_best["dgrad"] += dg * n
        row = dict(shape=f"N{N} {C}->{Co} k{k}s{s} {H}x{W}", count=n, fwd_us=fw, dgrad_us=dg,
                   wgrad_us=wg, fwd_tflops=flop / bf / 1e6, fwd_gbs=bytes_f / bf / 1e3,
                   wgrad_tflops=flop / bw / 1e6)
        rows.append(row)
        print(f"{row['shape']:34s} x{n}  fwd best {bf:7.1f}us ({row['fwd_tflops']:6.1f} TF, "
              f"{row['fwd_gbs']:6.0f} GB/s) v={min(fw, key=fw.get)} "
              f"| dgrad {dg or 0:7.1f}us | wgrad best {bw:7.1f}us ({row['wgrad_tflops']:6.1f} TF)"
              f" v={min(wg, key=wg.get)}", flush=True)
        print("    fwd us by variant: " + " ".join(f"{v}:{t:.0f}" for v, t in fw.items()) +
              " | wgrad: " + " ".join(f"{v}:{t:.0f}" for v, t in wg.items()), flush=True)
    print("totals (us, x count):", {k: round(v, 1) for k, v in tot_best.items()})
    if a.json:
        Path(a.json).write_text(json.dumps({"rows": rows, "totals_us": tot_best}, indent=1,
                                           default=str))


if __name__ == "__main__":
    main()
