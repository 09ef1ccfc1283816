"""Debug: every launch of the persistent 3x3 kernel (variant 20) inside a real training step is
re-run with the per-tile patch kernel (variant 15) into scratch outputs and compared."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("bench_main", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    from simclr_amd.ops import conv_hip
    import simclr_amd.models.fused as fused
    orig = conv_hip.igemm_launch

    def wrapped(ops, A, B, out, geom, v, *a, **kw):
        if v != 20:
            return orig(ops, A, B, out, geom, v, *a, **kw)
        stats = kw.get("stats")
        epi = kw.get("epi")
        mode = epi[0] if epi is not None else 0
        orig(ops, A, B, out, geom, v, *a, **kw)
        if mode not in (0, 3) or kw.get("tail") is not None:
            print("skip compare mode", mode, flush=True)
            return
        out2 = torch.empty_like(out)
        kw2 = dict(kw)
        if stats is not None:
            kw2["stats"] = torch.empty_like(stats)
        orig(ops, A, B, out2, geom, 15, *a, **kw2)
        torch.cuda.synchronize()
        d = (out.float() - out2.float()).abs().max().item()
        s = out2.float().abs().max().item()
        ds = ((stats - kw2["stats"]).abs().max().item() if stats is not None else 0.0)
        print(f"v20 mode {mode} M={geom[0]*geom[4]*geom[5]} out maxdiff {d:.3e} (max {s:.3e})"
              f" stats maxdiff {ds:.3e} nan={bool(torch.isnan(out).any())}", flush=True)

    conv_hip.igemm_launch = wrapped
    fused.igemm_launch = wrapped
    sys.argv = ["bench.py", "--steps", "2", "--warmup", "1", "--no-graph"]
    bench.main()


if __name__ == "__main__":
    main()
