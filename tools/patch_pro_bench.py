"""Patch kernels with vs without the BN-apply prologue at the ResNet-50 CIFAR conv2 shapes:
forward igemm_patch (PRO 1) and wgrad_patch (X prologue) against bn_apply_ss + plain kernel."""
import math
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])


def timeit(fn, reps=20):
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
    from simclr_amd.ops.conv_hip import fwd_geom
    ops = _ext.ops()
    dev = torch.device("cuda", 0)
    S, N = 2, 1024
    for H, C in ((32, 64), (16, 128)):
        M = N * H * H
        v = 15 if C == 64 else 16
        x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
        ss = torch.stack([torch.rand(S, C, device=dev) + 0.5,
                          torch.randn(S, C, device=dev) * 0.5]).reshape(2, S * C).contiguous()
        xb = torch.empty_like(x)
        w = (torch.randn(C, 3, 3, C, device=dev) / math.sqrt(9 * C)).to(torch.bfloat16)
        g = fwd_geom(N, H, H, C, H, H, 3, 3, 1, 1, C)
        out = torch.empty(N, H, H, C, device=dev, dtype=torch.bfloat16)
        t_apply = timeit(lambda: ops.bn_apply_ss(x, ss, None, None, xb, S, True))
        t_f0 = timeit(lambda: ops.igemm(xb, w, out, None, None, g, None, None, 0, False, 0, None,
                                        None, v))
        t_f1 = timeit(lambda: ops.igemm(x, w, out, None, None, g, ss[0], ss[1], M // S, True, 0,
                                        None, None, v))
        dy = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
        sp = ops.wgrad_splits(g, 17)
        part = torch.empty(sp * C * 9 * C, device=dev)
        o = torch.empty(C, 3, 3, C, device=dev)
        t_w0 = timeit(lambda: ops.wgrad(dy, xb, part, o, g, sp, C, 0.0, None, None, 0, False, 1, 17))
        t_w1 = timeit(lambda: ops.wgrad(dy, x, part, o, g, sp, C, 0.0, ss[0], ss[1], M // S, True,
                                        S, 17))
        print(f"H={H} C={C}: apply {t_apply:.1f} | fwd patch {t_f0:.1f} -> with prologue {t_f1:.1f}"
              f" | wgrad patch {t_w0:.1f} -> with prologue {t_w1:.1f} us", flush=True)
        if C == 64:  # persistent resident-weight kernel (variant 20)
            t_p0 = timeit(lambda: ops.igemm(xb, w, out, None, None, g, None, None, 0, False, 0,
                                            None, None, 20))
            t_p1 = timeit(lambda: ops.igemm(x, w, out, None, None, g, ss[0], ss[1], M // S, True,
                                            0, None, None, 20))
            st = torch.empty((M // 256) * 2 * C, device=dev)
            mi = torch.cat([torch.zeros(S, C, device=dev), torch.ones(S, C, device=dev)]).reshape(-1)
            sv = ss.reshape(-1)
            res = {}
            for v in (15, 20):
                res[v] = timeit(lambda: ops.igemm(xb, w, out, None, st, g, None, None, 0, False, 3,
                                                  None, x, v, sv, mi, M // S, 0, 0, None, None,
                                                  None, None, None, None, None))
            print(f"  persistent v20: fwd {t_p0:.1f} (v15 {t_f0:.1f}) | with prologue {t_p1:.1f}"
                  f" (v15 {t_f1:.1f}) | mode-3 dgrad epilogue v20 {res[20]:.1f} vs v15 "
                  f"{res[15]:.1f} us", flush=True)


if __name__ == "__main__":
    main()
