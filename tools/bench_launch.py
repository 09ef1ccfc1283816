"""Per-kernel dispatch cost on this GPU: a hipGraph of back-to-back tiny kernels (one of ours,
one torch elementwise) vs eager launches.  Usage (GPU box): python tools/bench_launch.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    from simclr_amd.ops import _ext
    _ext.require()
    ops = torch.ops.simclr_amd
    w = torch.zeros(8, 1, 1, 8, device="cuda", dtype=torch.bfloat16)
    wt = torch.empty_like(w)
    x = torch.zeros(8, device="cuda")
    n = 200

    def ours():
        for _ in range(n):
            ops.weight_transform(w, wt, [8, 1, 1, 8, 1, 1, 0, 1, 0, 1])

    def theirs():
        for _ in range(n):
            x.add_(1.0)
    for name, fn in (("simclr weight_transform", ours), ("torch add_", theirs)):
        eager = timed(fn, n)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        graph = timed(g.replay, n)
        print(f"{name:26s} eager {eager:6.2f} us/launch   graph {graph:6.2f} us/kernel")


if __name__ == "__main__":
    main()
