"""Per-entry-point config validation (``check_hydra_conf`` of the reference scripts,
SURVEY C4): main.py:39-50, eval.py:20-28 (momentum strictly > 0), save_features.py:15-17,
supervised.py:18-27.  Raises ``AssertionError`` with the failing key (the reference asserts)."""
from __future__ import annotations


def _check(cond: bool, msg: str) -> None:
    if not cond:
        raise AssertionError(msg)


def check_pretrain_conf(cfg) -> None:
    p, e = cfg["parameter"], cfg["experiment"]
    _check(p["temperature"] > 0.0, "parameter.temperature must be > 0")
    _check(p["epochs"] > 0, "parameter.epochs must be > 0")
    _check(e["batches"] > 0, "experiment.batches must be > 0")
    _check(1.0 > p["momentum"] >= 0, "parameter.momentum must be in [0, 1)")
    _check(p["warmup_epochs"] >= 0, "parameter.warmup_epochs must be >= 0")
    _check(p["d"] > 0, "parameter.d must be > 0")
    _check(e["base_cnn"] in {"resnet18", "resnet50"}, "experiment.base_cnn must be resnet18/50")
    _check(e["lr"] > 0.0, "experiment.lr must be > 0")
    _check(e["strength"] > 0.0, "experiment.strength must be > 0")
    _check(e["decay"] >= 0.0, "experiment.decay must be >= 0")


def check_eval_conf(cfg) -> None:
    p, e = cfg["parameter"], cfg["experiment"]
    _check(p["epochs"] > 0, "parameter.epochs must be > 0")
    _check(e["batches"] > 0, "experiment.batches must be > 0")
    _check(1.0 > p["momentum"] > 0.0, "parameter.momentum must be in (0, 1)")
    _check(p["warmup_epochs"] >= 0, "parameter.warmup_epochs must be >= 0")
    _check(e["base_cnn"] in {"resnet18", "resnet50"}, "experiment.base_cnn must be resnet18/50")
    _check(e["lr"] > 0.0, "experiment.lr must be > 0")
    _check(e["decay"] >= 0.0, "experiment.decay must be >= 0")


def check_save_features_conf(cfg) -> None:
    _check(cfg["parameter"]["epochs"] > 0, "parameter.epochs must be > 0")
    _check(cfg["experiment"]["base_cnn"] in {"resnet18", "resnet50"},
           "experiment.base_cnn must be resnet18/50")


def check_supervised_conf(cfg) -> None:
    p, e = cfg["parameter"], cfg["experiment"]
    _check(p["epochs"] > 0, "parameter.epochs must be > 0")
    _check(e["batches"] > 0, "experiment.batches must be > 0")
    _check(1.0 > p["momentum"] >= 0, "parameter.momentum must be in [0, 1)")
    _check(p["warmup_epochs"] >= 0, "parameter.warmup_epochs must be >= 0")
    _check(e["base_cnn"] in {"resnet18", "resnet50"}, "experiment.base_cnn must be resnet18/50")
    _check(e["lr"] > 0.0, "experiment.lr must be > 0")
    _check(e["strength"] > 0.0, "experiment.strength must be > 0")
    _check(e["decay"] >= 0.0, "experiment.decay must be >= 0")
