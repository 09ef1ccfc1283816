"""Probe: the ImageNet stem (7x7 / stride 2 / pad 3, 3 -> 64 channels) as run today (input
channels zero-padded to 8, K = 392) against its 2x2 space-to-depth form (a 4x4 / stride-1 conv over
the padded image folded to 12 -> 16 channels, K = 256), forward and weight gradient, every
admissible tile variant.  Usage (GPU box): python tools/stem_s2d_probe.py [N] [H]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from tools.conv_bench import timeit  # noqa: E402


def probe(ops, fwd_geom, N, H, C, k, s, p, Co, tag):
    dev = torch.device("cuda", 0)
    OH = (H + 2 * p - k) // s + 1
    x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
    w = (torch.randn(Co, k, k, C, device=dev) * 0.05).to(torch.bfloat16)
    y = torch.empty(N, OH, OH, Co, device=dev, dtype=torch.bfloat16)
    g = fwd_geom(N, H, H, C, OH, OH, k, k, s, p, Co)
    fw = {v: timeit(lambda v=v: ops.igemm(x, w, y, None, None, g, None, None, 0, False, 0, None,
                                          None, v))
          for v in range(ops.igemm_nvariants()) if ops.igemm_variant_ok(v, g, False, False)}
    dy = torch.randn(N, OH, OH, Co, device=dev).to(torch.bfloat16)
    out = torch.empty(Co, k, k, C, device=dev)
    wg = {}
    for v in range(ops.wgrad_nvariants()):
        if not ops.wgrad_variant_ok(v, g, False, False):
            continue
        sp = ops.wgrad_splits(g, v)
        part = torch.empty(sp * Co * k * k * C, device=dev)
        wg[v] = timeit(lambda v=v, sp=sp, part=part: ops.wgrad(dy, x, part, out, g, sp, C, 0.0,
                                                               None, None, 0, False, 1, v))
    bf, bw = min(fw, key=fw.get), min(wg, key=wg.get)
    print(f"{tag:28s} fwd best v{bf} {fw[bf]:8.1f} us | wgrad best v{bw} {wg[bw]:8.1f} us", flush=True)
    print("   fwd " + " ".join(f"{v}:{t:.0f}" for v, t in fw.items()), flush=True)
    print("   wgrad " + " ".join(f"{v}:{t:.0f}" for v, t in wg.items()), flush=True)
    del x, y, dy


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 224
    from simclr_amd.ops import _ext
    from simclr_amd.ops.conv_hip import fwd_geom
    ops = _ext.ops()
    probe(ops, fwd_geom, N, H, 8, 7, 2, 3, 64, "7x7/s2 C8 (today)")
    Hs = (H + 6) // 2
    probe(ops, fwd_geom, N, Hs, 16, 4, 1, 0, 64, "s2d 4x4/s1 C16")


if __name__ == "__main__":
    main()
