"""What a bf16 GEMM actually sustains on this MI355X, to price the convolutions against a
measured ceiling instead of the 2.5 PF/s datasheet number (the chip lowers its clock under a
dense MFMA load: MI355X guide, 'DVFS give-back').

Prints one markdown table: hipBLASLt (torch.matmul) bf16 GEMMs on random data at large shapes,
and this framework's LDS-DMA implicit GEMM (csrc/conv.hip igemm_glds) on the same shapes
expressed as a 1x1 convolution, best tile variant.  Usage (GPU box): python tools/mfma_ceiling.py
[MxNxK ...]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _time(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e-3


def main():
    from simclr_amd.ops import _ext
    from simclr_amd.ops.conv_hip import fwd_geom
    _ext.require()
    ops = torch.ops.simclr_amd
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    print("| M x N x K | hipBLASLt bf16 TF/s | igemm_glds best TF/s (variant) |")
    print("|---|---:|---:|")
    shapes = ((8192, 8192, 8192), (16384, 4096, 4096), (65536, 256, 2304),
              (262144, 128, 1152), (1048576, 64, 576))
    if len(sys.argv) > 1:  # e.g. 65536x1024x256 65536x256x1024
        shapes = [tuple(int(v) for v in a.split("x")) for a in sys.argv[1:]]
    for M, N, K in shapes:
        a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
        t = _time(lambda: torch.matmul(a, b))
        lib = 2.0 * M * N * K / t / 1e12
        # the same GEMM as a 1x1 convolution: [M, 1, 1, K] image, OHWI weight [N][K]
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        g = fwd_geom(M, 1, 1, K, 1, 1, 1, 1, 1, 0, N)
        best, bv = 0.0, -1
        for v in range(ops.igemm_nvariants()):
            if not ops.igemm_variant_glds(v) or not ops.igemm_variant_ok(v, g, False, False):
                continue
            if M % ops.igemm_variant_bm(v):
                continue
            tv = _time(lambda: ops.igemm(a, w, out, None, None, g, None, None, 0, False, 0, None,
                                         None, v, None, None, 0, 0, 0, None, None, None, None,
                                         None, None, None))
            tf = 2.0 * M * N * K / tv / 1e12
            if tf > best:
                best, bv = tf, v
        print(f"| {M} x {N} x {K} | {lib:.0f} | {best:.0f} ({bv}) |", flush=True)


if __name__ == "__main__":
    main()
