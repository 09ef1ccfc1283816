"""Microbenchmark of the memory-bound 1x1 convolutions of the ResNet-50 CIFAR step (layer1:
M = 1024*32*32 rows, K = 64 -> N = 256, and the dgrad direction with the mode-4 epilogue),
per tile variant and fusion, with achieved HBM bandwidth over the compulsory bytes.
Usage (GPU box): python tools/membound_bench.py [--rows 1048576] [--k 64] [--n 256]"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def timeit(fn, reps=10):
    fn()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1024 * 32 * 32)
    ap.add_argument("--k", type=int, default=64)
    ap.add_argument("--n", type=int, default=256)
    ap.add_argument("--only", type=int, default=-1, help="single variant (for profiling)")
    a = ap.parse_args()
    from simclr_amd.ops import _ext
    from simclr_amd.ops.conv_hip import fwd_geom
    ops = _ext.ops()
    dev = torch.device("cuda", 0)
    M, K, N, S = a.rows, a.k, a.n, 2
    img = M // 1024
    H = W = int(round(img ** 0.5))
    x = torch.randn(1024, H, W, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, 1, 1, K, device=dev) * 0.1).to(torch.bfloat16)
    y = torch.empty(1024, H, W, N, device=dev, dtype=torch.bfloat16)
    g = fwd_geom(1024, H, W, K, H, W, 1, 1, 1, 0, N)
    r = torch.randn_like(y)
    xa = torch.randn_like(y)
    mask = torch.randint(0, 255, (y.numel() // 8,), device=dev, dtype=torch.uint8)
    sc = torch.rand(S, K, device=dev) + 0.5
    sh = torch.randn(S, K, device=dev) * 0.1
    mi = torch.cat([torch.randn(S, N, device=dev) * 0.1, torch.rand(S, N, device=dev) + 0.5]).reshape(-1)
    base = 2.0 * (M * K + M * N)
    for v in range(ops.igemm_nvariants()):
        if (a.only >= 0 and v != a.only) or not ops.igemm_variant_ok(v, g, False, False):
            continue
        bm = ops.igemm_variant_bm(v)
        glds = ops.igemm_variant_glds(v)
        st = torch.empty((M // bm) * 2 * N, device=dev)
        res = {}
        res["epi0"] = (timeit(lambda: ops.igemm(x, w, y, None, None, g, None, None, 0, False, 0,
                                                 None, None, v)), base)
        res["epi0+st"] = (timeit(lambda: ops.igemm(x, w, y, None, st, g, None, None, 0, False, 0,
                                                    None, None, v)), base)
        if ops.igemm_variant_ok(v, g, True, False):
            res["pro+st"] = (timeit(lambda: ops.igemm(x, w, y, None, st, g, sc, sh, M // S, True,
                                                       0, None, None, v)), base)
        res["epi4+st"] = (timeit(lambda: ops.igemm(
            x, w, y, None, st, g, None, None, 0, False, 4, r, None, v, None, mi, M // S, 0, 0, xa,
            mask, None, None, None, None, None)), base + 4.0 * M * N + M * N / 8)
        print(f"v{v:2d} {bm}x{ops.igemm_variant_bn(v)}{' glds' if glds else ''}: " +
              "  ".join(f"{k} {t:6.1f}us {b / t / 1e6:5.2f}TB/s" for k, (t, b) in res.items()),
              flush=True)


if __name__ == "__main__":
    main()
