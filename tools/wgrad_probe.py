"""Run ONE weight-gradient launch configuration repeatedly (for rocprofv3 --pmc / kernel-trace
per-variant analysis).  Usage: python tools/wgrad_probe.py N C H Co k s p [variant|-1|v1,v2,..]
[reps] [rounds] — a list is timed in `rounds` interleaved rounds (box clock drift hits every arm);
variants the geometry does not admit are skipped."""
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main(N, C, H, Co, k, s, p, variant=-1, reps=20, rounds=1):
    from simclr_amd.ops import _ext
    from simclr_amd.ops.conv_hip import fwd_geom
    ops = _ext.ops()
    dev = torch.device("cuda", 0)
    OH = (H + 2 * p - k) // s + 1
    x = torch.randn(N, H, H, C, device=dev).to(torch.bfloat16)
    dy = torch.randn(N, OH, OH, Co, device=dev).to(torch.bfloat16)
    g = fwd_geom(N, H, H, C, OH, OH, k, k, s, p, Co)
    vs = (list(variant) if isinstance(variant, (list, tuple)) else
          [variant] if variant >= 0 else list(range(ops.wgrad_nvariants())))
    vs = [v for v in vs if ops.wgrad_variant_ok(v, g, False, False)]
    out = torch.empty(Co, k, k, C, device=dev)
    flop = 2.0 * N * OH * OH * Co * k * k * C
    for v in [v for _ in range(rounds) for v in vs]:
        sp = ops.wgrad_splits(g, v)
        part = torch.empty(sp * Co * k * k * C, device=dev)
        ops.wgrad(dy, x, part, out, g, sp, C, 0.0, None, None, 0, False, 1, v)
        torch.cuda.synchronize()
        st = torch.cuda.Event(enable_timing=True)
        en = torch.cuda.Event(enable_timing=True)
        st.record()
        for _ in range(reps):
            ops.wgrad(dy, x, part, out, g, sp, C, 0.0, None, None, 0, False, 1, v)
        en.record()
        en.synchronize()
        us = st.elapsed_time(en) / reps * 1e3
        print(f"variant {v:2d} splits {sp:3d}: {us:7.1f} us  {flop / us / 1e6:7.1f} TF/s",
              flush=True)


if __name__ == "__main__":
    a = [[int(x) for x in v.split(",")] if "," in v else int(v) for v in sys.argv[1:]]
    main(*a)
