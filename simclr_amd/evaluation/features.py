"""Feature extraction from a pre-trained ContrastiveModel, and the eval / save_features drivers.

Reference: ``convert_vectors`` (``/root/reference/eval.py:31-58``; save_features.py:20-77) —
``model.eval()``, ``no_grad``, ``encode(x)`` (h) or ``forward(x)`` (z) per
``parameter.use_full_encoder``; the eval driver (eval.py:193-325) loops over
``target_dir/*.pt``, strips ``module.``, loads ``strict=False``, extracts train/val features
from un-augmented data (ToTensor only) and runs the selected probe, writing ``results.json``
keyed by checkpoint file name.  ``save_features`` (save_features.py:119-179) writes
``{key}.feature.{train,val}.npy`` / ``{key}.label.{train,val}.npy`` and the means of 1/5/20
augmented passes ``{key}.aug-{t}.feature.{train,val}.npy`` (strength 0.5, view 0).

Fixed defects: eval.py's invalid ``load_state_dict(map_location=...)`` (Q3) and save_features'
missing ``module.`` strip (Q5); ``model.g[-1]`` / ``model.g[0]`` (Q2) are replaced by the head's
``out_features`` / ``in_features``.  Relative ``target_dir`` is resolved against the launch
directory (the run directory is the cwd under Hydra semantics).
"""
from __future__ import annotations

import json
import logging
from pathlib import Path
from typing import List, Optional, Tuple

import numpy as np
import torch

from ..config import check_eval_conf, check_save_features_conf, to_absolute_path
from ..data.datasets import load_dataset
from ..data.loader import ContrastiveLoader, EvalLoader
from ..models.contrastive import ContrastiveModel
from ..ops import registry
from ..parallel.flat import FlatParamStore
from ..runtime.dist import pick_device
from ..utils.checkpoint import load_into
from ..utils.misc import cfg_get, seed_everything
from .probes import DownstreamDataset, run_probe

log = logging.getLogger(__name__)


def build_eval_model(cfg, device, precision: str, ckpt: Optional[Path] = None):
    model = ContrastiveModel(base_cnn=cfg["experiment"]["base_cnn"], d=cfg["parameter"]["d"],
                             cifar_stem=cfg_get(cfg, "model.cifar_stem", None),
                             stem_padding=cfg_get(cfg, "model.stem_padding", 3)).to(device)
    shadow = torch.bfloat16 if (precision == "bf16" and device.type == "cuda") else None
    store = FlatParamStore(model, device, shadow_dtype=shadow)
    if ckpt is not None:
        missing, unexpected = load_into(model, ckpt, strict=False, store=store)
        if unexpected:
            log.warning("unexpected keys in %s: %s", ckpt, unexpected[:5])
    model.eval()
    return model, store


def _prep(x: torch.Tensor, precision: str, device) -> torch.Tensor:
    if precision == "bf16" and device.type == "cuda":
        return x
    x = x.float()
    return (x[:, :3] if x.shape[1] != 3 else x).contiguous()


@torch.no_grad()
def convert_vectors(model, loader, use_full_encoder: bool, precision: str,
                    device) -> Tuple[torch.Tensor, torch.Tensor]:
    xs, ys = [], []
    for x, y in loader:
        x = _prep(x, precision, device)
        f = model(x) if use_full_encoder else model.encode(x)
        xs.append(f.float())
        ys.append(y)
    return torch.cat(xs), torch.cat(ys)


def _datasets(cfg):
    seed = cfg["parameter"]["seed"]
    kw = dict(root=cfg_get(cfg, "data.root", "~/pytorch_datasets"),
              synthetic=bool(cfg_get(cfg, "data.synthetic", False)),
              allow_synthetic_fallback=bool(cfg_get(cfg, "data.synthetic_fallback", False)),
              synthetic_noise=float(cfg_get(cfg, "data.synthetic_noise", 25.0)),
              synthetic_colour=bool(cfg_get(cfg, "data.synthetic_colour", True)),
              synthetic_kind=str(cfg_get(cfg, "data.synthetic_kind", "template")),
              seed=seed)
    size = cfg_get(cfg, "data.synthetic_size", None)
    tr = load_dataset(cfg["experiment"]["name"], train=True,
                      synthetic_size=size, **kw)
    va = load_dataset(cfg["experiment"]["name"], train=False,
                      synthetic_size=(max(1, size // 5) if size else None), **kw)
    return tr, va


def _setup(cfg):
    seed_everything(cfg["parameter"]["seed"])
    use_cuda = cfg["parameter"]["use_cuda"] and torch.cuda.is_available()
    device = pick_device(0, use_cuda)
    registry.set_backend(cfg_get(cfg, "runtime.backend", "auto"))
    precision = cfg_get(cfg, "runtime.precision", "bf16") if device.type == "cuda" else "fp32"
    logging.info("Using {}".format(device))
    return device, precision


def checkpoints(target_dir: str) -> List[Path]:
    return sorted(Path(to_absolute_path(str(target_dir))).glob("*.pt"))


def evaluate(cfg) -> dict:
    check_eval_conf(cfg)
    device, precision = _setup(cfg)
    tr, va = _datasets(cfg)
    num_classes = tr.num_classes
    bs = cfg["experiment"]["batches"]
    top_k = cfg["parameter"]["top_k"]
    full = bool(cfg["parameter"]["use_full_encoder"])
    results = {}
    for path in checkpoints(cfg["experiment"]["target_dir"]):
        if path.name.startswith("resume-"):
            continue
        key = path.name
        logging.info("Evaluation by using {}".format(key))
        model, _store = build_eval_model(cfg, device, precision, path)
        Xtr, ytr = convert_vectors(model, EvalLoader(tr, bs, device), full, precision, device)
        Xva, yva = convert_vectors(model, EvalLoader(va, bs, device), full, precision, device)
        results[key] = run_probe(cfg, cfg["parameter"]["classifier"], DownstreamDataset(Xtr, ytr),
                                 DownstreamDataset(Xva, yva), num_classes, top_k, device)
    with open(cfg["parameter"]["classification_results_json_fname"], "w") as f:
        json.dump(results, f)
    return results


def save_features(cfg) -> List[str]:
    check_save_features_conf(cfg)
    device, precision = _setup(cfg)
    tr, va = _datasets(cfg)
    bs = cfg["experiment"]["batches"]
    full = bool(cfg["parameter"]["use_full_encoder"])
    written = []
    for path in checkpoints(cfg["experiment"]["target_dir"]):
        if path.name.startswith("resume-"):
            continue
        key = path.name
        logging.info("Save features extracted by using {}".format(key))
        model, _store = build_eval_model(cfg, device, precision, path)
        for split, ds in (("train", tr), ("val", va)):
            X, y = convert_vectors(model, EvalLoader(ds, bs, device), full, precision, device)
            for kind, arr in (("feature", X), ("label", y)):
                fn = "{}.{}.{}.npy".format(key, kind, split)
                np.save(fn, arr.cpu().numpy())
                written.append(fn)
        # averages of augmented view-0 features over 1 / 5 / 20 passes (strength 0.5)
        sizes = (1, 5, 20)
        sums = {"train": None, "val": None}
        for t in range(1, sizes[-1] + 1):
            for split, ds in (("train", tr), ("val", va)):
                ld = ContrastiveLoader(ds, bs, device, views=1, strength=0.5,
                                       seed=cfg["parameter"]["seed"], shuffle=False,
                                       drop_last=False)
                ld.counter = t * 1000003
                X, _ = convert_vectors(model, ld, full, precision, device)
                sums[split] = X if sums[split] is None else sums[split] + X
                if t in sizes:
                    fn = "{}.aug-{}.feature.{}.npy".format(key, t, split)
                    np.save(fn, (sums[split] / t).cpu().numpy())
                    written.append(fn)
    return written
