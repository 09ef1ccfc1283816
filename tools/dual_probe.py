"""Time the fused 1x1 backward kernels (conv1x1_bwd_dual) on their production shapes, alone:
the narrow 8-wave form (layer1 conv3: Co 256 / Ci 64, 2^20 rows, lazy BN3 prologue), the wide
form (layer2 conv3: Co 512 / Ci 128, 2^18 rows, lazy, X materialised or BN2-applied in the
kernel) and the plain narrow form (layer1.0 downsample).  Prints us and the compulsory-byte
bandwidth.  Usage (GPU box): python tools/dual_probe.py [reps]"""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main(reps=20):
    from simclr_amd.ops import _ext
    ops = _ext.ops()
    dev = torch.device("cuda", 0)
    S = 2

    def bf(t):
        return t.to(torch.bfloat16)

    cases = [("narrow layer1 conv3 (lazy, dual8)", 1024, 32, 256, 64, True, False, False, 128, True),
             ("plain layer1.0 ds (lazy, dual8)", 1024, 32, 256, 64, True, False, True, 128, True),
             ("wide layer2 conv3 (lazy, X pre)", 1024, 16, 512, 128, True, True, False, 64, False),
             ("wide layer2 conv3 (lazy, X bn2)", 1024, 16, 512, 128, True, False, False, 64, False)]
    for name, Nb, H, Co, Ci, lazy, pre, plain, bps, dual8 in cases:
        M = Nb * H * H
        G = bf(torch.randn(M, Co, device=dev))
        A3 = bf(torch.randn(M, Co, device=dev)) if lazy else None
        coef = (torch.randn(3 * S * Co, device=dev) * 0.5) if lazy else None
        X = bf(torch.randn(M, Ci, device=dev))
        ss = torch.cat([0.5 + torch.rand(S * Ci, device=dev), torch.randn(S * Ci, device=dev) * 0.3])
        mi = torch.cat([torch.randn(S * Ci, device=dev) * 0.1, 0.5 + torch.rand(S * Ci, device=dev)])
        Wt = bf(torch.randn(Ci, Co, device=dev) * 0.04)
        gm = torch.empty(M, Ci, device=dev, dtype=torch.bfloat16)
        stats = torch.empty(S * bps * 2 * Ci, device=dev)
        wpart = torch.empty(S * bps * Co * Ci, device=dev)
        Xp = bf(torch.relu(X.float())) if pre else None

        def run():
            if plain:
                ops.conv1x1_bwd_dual(G, A3, coef, X, None, None, Wt, gm, stats, wpart, S, bps,
                                     None, dual8)
            else:
                ops.conv1x1_bwd_dual(G, A3, coef, Xp if pre else X, ss, mi, Wt, gm, stats, wpart,
                                     S, bps, X if pre else None, dual8)
        run()
        torch.cuda.synchronize()
        st, en = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(reps):
            run()
        en.record()
        en.synchronize()
        us = st.elapsed_time(en) / reps * 1e3
        nbytes = 2 * M * Co * (2 if lazy else 1) + 2 * M * Ci * (3 if pre else 2) + 4 * wpart.numel()
        print(f"{name:36s} {us:8.1f} us  {nbytes / us / 1e6:6.2f} TB/s (compulsory {nbytes / 1e6:.0f} MB)",
              flush=True)
        del G, A3, X, gm, wpart, Xp


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
