"""Short-K 1x1 conv GEMMs of the ResNet-50 bottleneck (conv3 expansion forward C -> 4C with the
BN2-apply prologue, conv1 reduction 4C -> C) per tile variant, with BatchNorm statistics
partials, at the executor's shapes (1024 rows of images = 512 x 2 views, 2 BN segments).
Usage: python tools/shortk_bench.py [--no-pro]"""
import math
import sys

import torch

sys.path.insert(0, "/root/repo")
from simclr_amd.ops import _ext  # noqa: E402
from simclr_amd.ops.conv_hip import fwd_geom  # noqa: E402

ops = _ext.ops()
dev = torch.device("cuda", 0)


def timeit(fn, reps=20):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


S = 2
SHAPES = [  # (images, H, Cin, Cout, prologue)
    (1024, 32, 64, 256, True), (1024, 16, 128, 512, True), (1024, 8, 256, 1024, True),
    (1024, 4, 512, 2048, True), (1024, 32, 256, 64, True), (1024, 16, 512, 128, True),
    (1024, 8, 1024, 256, True), (1024, 4, 2048, 512, True)]
use_pro = "--no-pro" not in sys.argv
for (N, H, C, Co, pro) in SHAPES:
    pro = pro and use_pro
    M = N * H * H
    x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
    w = (torch.randn(Co, 1, 1, C, device=dev) / math.sqrt(C)).to(torch.bfloat16)
    y = torch.empty(N, H, H, Co, device=dev, dtype=torch.bfloat16)
    sc = torch.rand(S, C, device=dev) + 0.5
    sh = torch.randn(S, C, device=dev) * 0.1
    g = fwd_geom(N, H, H, C, H, H, 1, 1, 1, 0, Co)
    res = []
    for v in range(ops.igemm_nvariants()):
        if not ops.igemm_variant_ok(v, g, pro, False):
            continue
        bm = ops.igemm_variant_bm(v)
        if (M // S) % bm:
            continue
        st = torch.empty((M // bm) * 2 * Co, device=dev)
        if pro:
            t = timeit(lambda: ops.igemm(x, w, y, None, st, g, sc, sh, M // S, True, 0, None, None,
                                         v))
        else:
            t = timeit(lambda: ops.igemm(x, w, y, None, st, g, None, None, 0, False, 0, None, None,
                                         v))
        res.append((v, t))
    fl = 2.0 * M * Co * C
    by = 2.0 * (M * C + M * Co)
    best = min(res, key=lambda r: r[1])
    print(f"M={M} N={Co} K={C} pro={int(pro)}: best v{best[0]} {best[1]:.1f} us "
          f"({fl / best[1] / 1e6:.0f} TF/s, {by / best[1] / 1e3:.0f} GB/s)  all: "
          + " ".join(f"v{v}:{t:.0f}" for v, t in res), flush=True)
