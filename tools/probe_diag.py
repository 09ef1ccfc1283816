"""Feature diagnostics behind a linear-probe number (profiles/r3_e2e_probe_diag.md).

For every reference-format checkpoint in a run directory: extract the encoder features h of the
train / val splits exactly as eval.py does (``evaluation.features``), then report
  * scale: mean / max row norm, NaN / Inf count, per-dimension std (min / median / max);
  * collapse: effective rank exp(H(σ²/Σσ²)) of the centred train features, and the share of the
    variance in the top singular direction;
  * probes: the reference linear probe (eval.py:88-190 semantics, ``run_probe``) on the raw
    features — train AND val accuracy — the same probe on standardised features (train mean /
    std), and the centroid probe.
A probe that fails on raw features but works on standardised ones is an optimisation (scale)
problem; one that fails on both while the train accuracy is also at chance means the features
carry no class information.

Usage: python tools/probe_diag.py RUN_DIR [hydra overrides of eval.yaml ...]
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))


def stats(X: torch.Tensor) -> dict:
    X = X.float()
    finite = torch.isfinite(X)
    Xf = torch.where(finite, X, torch.zeros_like(X))
    nrm = Xf.norm(dim=1)
    sd = Xf.std(dim=0)
    Xc = (Xf - Xf.mean(0, keepdim=True)).double()
    sv = torch.linalg.svdvals(Xc[: min(20000, Xc.shape[0])])
    p = sv ** 2 / (sv ** 2).sum().clamp_min(1e-30)
    ent = -(p * torch.log(p.clamp_min(1e-30))).sum()
    return {"row_norm_mean": float(nrm.mean()), "row_norm_max": float(nrm.max()),
            "nonfinite": int((~finite).sum()), "dim_std_min": float(sd.min()),
            "dim_std_median": float(sd.median()), "dim_std_max": float(sd.max()),
            "effective_rank": float(torch.exp(ent)), "top_sv_share": float(p[0]),
            "dims": int(X.shape[1])}


def main(argv):
    from simclr_amd.config import compose, task_config, CONF_DIR
    from simclr_amd.data.loader import EvalLoader
    from simclr_amd.evaluation.features import (_datasets, _setup, build_eval_model,
                                                checkpoints, convert_vectors)
    from simclr_amd.evaluation.probes import DownstreamDataset, run_probe
    run_dir, ov = argv[0], argv[1:]
    cfg = task_config(compose(str(CONF_DIR), "eval", ov + [f"experiment.target_dir={run_dir}"],
                              job_name="probe_diag"))
    device, precision = _setup(cfg)
    tr, va = _datasets(cfg)
    bs = cfg["experiment"]["batches"]
    out = {}
    for path in checkpoints(run_dir):
        if path.name.startswith("resume-"):
            continue
        model, _ = build_eval_model(cfg, device, precision, path)
        Xtr, ytr = convert_vectors(model, EvalLoader(tr, bs, device), False, precision, device)
        Xva, yva = convert_vectors(model, EvalLoader(va, bs, device), False, precision, device)
        rec = {"train_features": stats(Xtr)}
        mu, sd = Xtr.mean(0, keepdim=True), Xtr.std(0, keepdim=True).clamp_min(1e-6)
        for name, (a, b) in {"raw": (Xtr, Xva),
                             "standardised": ((Xtr - mu) / sd, (Xva - mu) / sd)}.items():
            r = run_probe(cfg, "linear", DownstreamDataset(a, ytr), DownstreamDataset(b, yva),
                          tr.num_classes, cfg["parameter"]["top_k"], device)
            rec[f"linear_{name}"] = {"train_acc_last": r["train_accuracies"][-1],
                                     "val_acc_best": r["highest_val_acc"],
                                     "train_loss_last": r["train_losses"][-1]}
        c = run_probe(cfg, "centroid", DownstreamDataset(Xtr, ytr), DownstreamDataset(Xva, yva),
                      tr.num_classes, cfg["parameter"]["top_k"], device)
        rec["centroid"] = {"train_acc": c["train_acc"], "val_acc": c["val_acc"]}
        out[path.name] = rec
        print(path.name, json.dumps(rec), flush=True)
    return out


if __name__ == "__main__":
    main(sys.argv[1:])
