"""Per-variant time of the 1x1 dgrad with the BN-backward operand prologue (PRO 2) at the
ResNet-50 CIFAR conv3 shapes, against materialising da first (bn_bwd_apply + plain dgrad)."""
import math
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])


def timeit(fn, reps=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    from simclr_amd.ops import _ext
    ops = _ext.ops()
    dev = torch.device("cuda", 0)
    S = 2
    for (N, H, Ci, Co) in [(1024, 32, 64, 256), (1024, 16, 128, 512), (1024, 8, 256, 1024)]:
        M = N * H * H
        g = torch.randn(N, H, H, Co, device=dev).to(torch.bfloat16)
        a = torch.randn(N, H, H, Co, device=dev).to(torch.bfloat16)
        coef = torch.randn(3 * S * Co, device=dev) * 0.5
        wt = (torch.randn(Ci, Co, device=dev) / math.sqrt(Co)).to(torch.bfloat16)
        geom = [N, H, H, Co, H, H, 1, 1, 1, 1, 1, 1, 0, 0, Ci, H, H, 1, 1, 0, 0, Ci]
        out = torch.empty(N, H, H, Ci, device=dev, dtype=torch.bfloat16)
        da = torch.empty_like(a)
        c = coef.view(3, S * Co)
        t_apply = timeit(lambda: ops.bn_bwd_apply(g, None, a, coef, S, False, da, None))
        plain = {v: timeit(lambda: ops.igemm(da, wt, out, None, None, geom, None, None, 0, False,
                                             0, None, None, v))
                 for v in range(ops.igemm_nvariants()) if ops.igemm_variant_ok(v, geom, False, False)}
        pro = {}
        for v in range(ops.igemm_nvariants()):
            if not ops.igemm_variant_ok(v, geom, True, True) or (M // S) % ops.igemm_variant_bm(v):
                continue
            pro[v] = timeit(lambda: ops.igemm(g, wt, out, None, None, geom, c[0], c[1], M // S,
                                              False, 0, None, None, v, None, None, 0, 0, 0, None,
                                              None, None, None, None, c[2], a, None, None, None))
        bp = min(plain, key=plain.get)
        print(f"M={M} N={Ci} K={Co}: materialise {t_apply:.0f} + dgrad {plain[bp]:.0f} (v{bp}) = "
              f"{t_apply + plain[bp]:.0f} us | prologue: " +
              " ".join(f"v{v}{'g' if ops.igemm_variant_glds(v) else ''}:{t:.0f}" for v, t in pro.items()),
              flush=True)


if __name__ == "__main__":
    main()
