"""Per-op timing of one SimCLR training step with semantic labels (conv shape / pass / fusion
mode), using HIP events around every ``torch.ops.simclr_amd`` call.

Usage (GPU box): python tools/layer_profile.py [--batch 512] [--steps 3] > out.md
Every op is bracketed by events on the current stream (no extra synchronisation inside the
step), so the numbers are the kernels' own durations in their real order."""
import argparse
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _Timed:
    def __init__(self, real, log):
        self._real = real
        self._log = log

    def __getattr__(self, name):
        f = getattr(self._real, name)
        if not callable(f) or "variant" in name or name.endswith(("_bm", "_bn", "splits", "blocks", "_ok")):
            return f

        def wrap(*args, **kw):
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
            r = f(*args, **kw)
            e.record()
            from simclr_amd.ops import _ext as ext
            lab, fl, by = _label(name, args)
            self._log.append(((lab, fl, by, ext.TAG), s, e))
            return r
        return wrap


def _nb(t):
    return t.numel() * t.element_size() if isinstance(t, torch.Tensor) else 0


def _label(name, args):
    """(label, flops, compulsory bytes): every operand read or written once (HBM roofline)."""
    if name == "igemm":
        g = args[5]
        M = g[0] * g[4] * g[5]
        K = g[6] * g[7] * g[3]
        mode = args[10] if len(args) > 10 else 0
        pro = args[6] is not None
        kind = "fwd" if g[10] == 1 and g[12] <= 0 and g[17] == 1 else "dgrad"
        extra = [args[i] for i in (11, 12, 19, 20, 21, 25, 27, 28) if len(args) > i]
        byts = _nb(args[0]) + _nb(args[1]) + 2 * M * g[14] + sum(_nb(t) for t in extra)
        fus = (" bnb" if len(args) > 24 and args[24] is not None else "") + \
              (" dual" if len(args) > 27 and args[27] is not None else "")
        return (f"igemm {kind} M={M} N={g[14]} K={K} k={g[6]} s={g[8]}{' pro' if pro else ''}"
                f"{fus} epi{mode & 255}", 2.0 * M * g[14] * K, byts)
    if name == "wgrad":
        g = args[4]
        M = g[0] * g[4] * g[5]
        K = g[6] * g[7] * g[3]
        splits = args[5]
        byts = _nb(args[0]) + _nb(args[1]) + 2 * 4 * splits * g[14] * K + _nb(args[3])
        if len(args) > 14:
            byts += _nb(args[14])
        return (f"wgrad M={M} N={g[14]} K={K} k={g[6]}{' pro' if args[8] is not None else ''}",
                2.0 * M * g[14] * K, byts)
    shape = tuple(args[0].shape) if hasattr(args[0], "shape") else ""
    return f"{name} {shape}", 0.0, sum(_nb(t) for t in args)


PEAK_FLOPS = 2.5e15   # bf16 dense MFMA peak (no sparsity)
PEAK_BYTES = 6.3e12   # achievable HBM3E stream bandwidth (MI355X_MICROARCH.md: float4 copy)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--size", type=int, default=32)
    ap.add_argument("--reference-stem", dest="cifar_stem", action="store_false", default=True,
                    help="the reference's stem (r50: ImageNet 7x7/s2 + maxpool)")
    ap.add_argument("--model", default="resnet50")
    a = ap.parse_args()
    from simclr_amd.ops import _ext
    from simclr_amd.config import compose, task_config, CONF_DIR
    from simclr_amd.data.datasets import synthetic_dataset
    from simclr_amd.data.loader import ContrastiveLoader
    from simclr_amd.parallel import state as pstate
    from simclr_amd.train.pretrain import Trainer
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    st = pstate.get()
    st.device = dev
    cfg = task_config(compose(str(CONF_DIR), "config", [
        f"experiment.base_cnn={a.model}", f"model.cifar_stem={'true' if a.cifar_stem else 'null'}",
        f"experiment.batches={a.batch}", "data.synthetic=true", "parameter.epochs=10"]))
    tr = Trainer(cfg, st, 50000)
    loader = ContrastiveLoader(synthetic_dataset(max(2048, (3 + a.steps) * a.batch), 10, size=a.size), a.batch,
                               dev, seed=7)
    it = iter(loader)
    for _ in range(2):  # warm-up + autotune
        tr.step(next(it)[0])
    torch.cuda.synchronize()
    log = []
    real = _ext.ops()
    timed = _Timed(real, log)
    _ext.ops = lambda: timed
    for _ in range(a.steps):
        tr.step(next(it)[0])
    torch.cuda.synchronize()
    agg = defaultdict(lambda: [0, 0.0, 0.0, 0.0])
    by_tag = defaultdict(float)
    fam = defaultdict(lambda: [0.0, 0.0])  # kernel family -> [us, ideal us]
    for (lab, flops, byts, tag), s, e in log:
        v = agg[lab]
        v[0] += 1
        t = s.elapsed_time(e) * 1e3
        v[1] += t
        v[2] += flops
        v[3] += byts
        ideal = max(flops / PEAK_FLOPS, byts / PEAK_BYTES) * 1e6
        f = fam[lab.split(" ")[0] + (" " + lab.split(" ")[1] if lab.startswith("igemm") else "")]
        f[0] += t
        f[1] += ideal
        # aggregate blocks of the same stage: "layer1.2 conv3 dgrad" -> "layer1 conv3 dgrad"
        parts = tag.split(" ")
        if parts and parts[0].startswith("layer"):
            parts[0] = parts[0].split(".")[0] + (".0" if parts[0].endswith(".0") else ".x")
        by_tag[" ".join(parts) or "(stem/head/loss/optim)"] += t
    tot = sum(v[1] for v in agg.values()) / a.steps
    print(f"# per-op time, {a.model} {'CIFAR' if a.cifar_stem else 'reference'} stem, {a.size}x{a.size}, "
          f"batch {a.batch}x2 views, avg of {a.steps} steps\n")
    print(f"total timed op time/step: {tot / 1e3:.2f} ms\n")
    print("roofline per op: max(FLOP / 2.5 PF/s bf16 dense, compulsory bytes / 6.3 TB/s); "
          "% = roofline time / measured time; bound = which term dominates\n")
    print("| op | calls/step | us/step | % of step | TF/s | TB/s | bound | % roofline |\n"
          "|---|---:|---:|---:|---:|---:|---|---:|")
    for lab, (n, t, fl, by) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        sec = t * 1e-6
        tf = f"{fl / sec / 1e12:.0f}" if fl else ""
        tb = f"{by / sec / 1e12:.2f}"
        ideal = max(fl / PEAK_FLOPS, by / PEAK_BYTES)
        bound = "MFMA" if fl / PEAK_FLOPS > by / PEAK_BYTES else "HBM"
        print(f"| {lab} | {n / a.steps:.1f} | {t / a.steps:.1f} | {100 * t / a.steps / tot:.1f} "
              f"| {tf} | {tb} | {bound} | {100 * ideal / sec:.0f} |")
    print("\n## by kernel family\n")
    print("| family | us/step | roofline us/step | % roofline |\n|---|---:|---:|---:|")
    for k, (t, ideal) in sorted(fam.items(), key=lambda kv: -kv[1][0]):
        print(f"| {k} | {t / a.steps:.1f} | {ideal / a.steps:.1f} | {100 * ideal / t:.0f} |")
    from simclr_amd.ops import tuning
    print("\n## autotuned tile variants (key -> variant)\n")
    ops = real
    for key, v in sorted(tuning.table().items(), key=lambda kv: str(kv[0])):
        if key[0] == "igemm":
            g = key[1]
            desc = f"M={g[0] * g[4] * g[5]} N={g[14]} K={g[6] * g[7] * g[3]} epi{key[4]}{' pro' if key[3] else ''}"
            tile = f"{ops.igemm_variant_bm(v)}x{ops.igemm_variant_bn(v)}"
        else:
            g = key[1]
            desc = f"wgrad M={g[0] * g[4] * g[5]} N={g[14]} K={g[6] * g[7] * g[3]}{' pro' if key[3] else ''}"
            tile = f"v{v}"
        print(f"- {key[0]} {desc}: {tile}")
    print("\n## by executor stage / op (layerN.0 = first block, layerN.x = the rest)\n")
    print("| stage op | us/step | % |\n|---|---:|---:|")
    for k, t in sorted(by_tag.items(), key=lambda kv: -kv[1]):
        print(f"| {k} | {t / a.steps:.1f} | {100 * t / a.steps / tot:.1f} |")


if __name__ == "__main__":
    main()
