"""Tiny driver for counter runs of the layer1 3x3 patch kernels (per-tile v15 vs persistent v20),
forward with and without the BN-apply prologue and the mode-3 dgrad epilogue: 3 launches each."""
import math
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])


def main():
    from simclr_amd.ops import _ext
    from simclr_amd.ops.conv_hip import fwd_geom
    ops = _ext.ops()
    dev = torch.device("cuda", 0)
    S, N, H, C = 2, 1024, 32, 64
    M = N * H * H
    x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
    xb = torch.relu(x)
    ss = torch.stack([torch.rand(S, C, device=dev) + 0.5,
                      torch.randn(S, C, device=dev) * 0.5]).reshape(2, S * C).contiguous()
    w = (torch.randn(C, 3, 3, C, device=dev) / math.sqrt(9 * C)).to(torch.bfloat16)
    g = fwd_geom(N, H, H, C, H, H, 3, 3, 1, 1, C)
    out = torch.empty(N, H, H, C, device=dev, dtype=torch.bfloat16)
    st = torch.empty((M // 256) * 2 * C, device=dev)
    mi = torch.cat([torch.zeros(S, C, device=dev), torch.ones(S, C, device=dev)]).reshape(-1)
    for v in (15, 20):
        for _ in range(3):
            ops.igemm(xb, w, out, None, None, g, None, None, 0, False, 0, None, None, v)
            ops.igemm(x, w, out, None, None, g, ss[0], ss[1], M // S, True, 0, None, None, v)
            ops.igemm(xb, w, out, None, st, g, None, None, 0, False, 3, None, x, v, ss.reshape(-1),
                      mi, M // S, 0, 0, None, None, None, None, None, None, None)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
