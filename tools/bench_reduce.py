"""Micro-benchmark of the one-launch BatchNorm partial reduction (``bn_reduce_fused``) on the
partial-array shapes of the ResNet-50 CIFAR step (batch 512x2): per-call time from a hipGraph
of back-to-back launches (no launch overhead), per (C, blocks-per-segment).

Usage (GPU box): python tools/bench_reduce.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [(64, 4096), (256, 4096), (128, 2048), (128, 1024), (512, 1024), (256, 256),
          (1024, 256), (512, 64), (2048, 64), (2048, 128)]


def main():
    from simclr_amd.ops import _ext
    _ext.require()
    ops = torch.ops.simclr_amd
    S, reps = 2, 50

    for C, nblk in SHAPES:
        part = torch.randn(S * nblk * 2 * C, device="cuda")
        mi = torch.empty(2 * S * C, device="cuda")
        ss = torch.empty(2 * S * C, device="cuda")
        rm = torch.zeros(C, device="cuda")
        rv = torch.ones(C, device="cuda")
        gam = torch.ones(C, device="cuda")
        bet = torch.zeros(C, device="cuda")

        def call():
            ops.bn_reduce_fused(part, nblk, S, C, 1, None, float(nblk * 128), 1e-5, 0.1, rm, rv,
                                mi, None, gam, bet, ss, None, None, None)
        call()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                call()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(4):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / (4 * reps)
        mb = part.numel() * 4 / 1e6
        print(f"C={C:5d} nblk={nblk:5d} partial={mb:6.2f} MB  {us:6.2f} us  {mb / us:.2f} TB/s")


if __name__ == "__main__":
    main()
