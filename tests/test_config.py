"""Hydra-compatible composer: the reference's YAML tree must load unchanged."""
import datetime
from pathlib import Path

import pytest

from simclr_amd.config import (CONF_DIR, ConfigCompositionError, compose, hydra_main, parse_value,
                               task_config)

REF_CONF = Path("/root/reference/conf")


def test_repo_config_defaults():
    cfg = task_config(compose(str(CONF_DIR), "config"))
    assert cfg["parameter"]["seed"] == 7
    assert cfg["parameter"]["temperature"] == 0.5
    assert cfg.experiment.decay == pytest.approx(1e-4) and isinstance(cfg.experiment.decay, float)
    assert cfg.experiment.batches == 512
    assert cfg.experiment.base_cnn == "resnet18"
    assert cfg.distributed.world_size == 4
    assert cfg.distributed.dist_url == "env://"
    assert cfg.loss.gather is False
    assert "hydra" not in cfg


@pytest.mark.skipif(not REF_CONF.exists(), reason="reference tree not mounted")
@pytest.mark.parametrize("name", ["config", "eval", "supervised_config"])
def test_reference_yaml_loads_unchanged(name):
    ref = task_config(compose(str(REF_CONF), name))
    ours = task_config(compose(str(CONF_DIR), name))
    # every reference key exists with the same value in our tree
    def walk(a, b, path=""):
        for k, v in a.items():
            assert k in b, f"missing key {path}{k}"
            if isinstance(v, dict):
                walk(v, b[k], f"{path}{k}.")
            else:
                assert b[k] == v, f"{path}{k}: {b[k]!r} != {v!r}"
    walk(ref, ours)


def test_overrides_and_struct_mode():
    cfg = task_config(compose(str(CONF_DIR), "config", [
        "parameter.epochs=3", "experiment.lr=0.5", "+foo.bar=[1,2]", "experiment=cifar100",
        "runtime.max_steps=null"]))
    assert cfg.parameter.epochs == 3
    assert cfg.experiment.name == "cifar100"
    assert cfg.experiment.lr == 0.5  # value override applies after group selection
    assert cfg.foo.bar == [1, 2]
    assert cfg.runtime.max_steps is None
    with pytest.raises(ConfigCompositionError):
        compose(str(CONF_DIR), "config", ["parameter.nonexistent=1"])
    with pytest.raises(ConfigCompositionError):
        compose(str(CONF_DIR), "config", ["+parameter.seed=1"])
    cfg = task_config(compose(str(CONF_DIR), "config", ["++parameter.seed=11", "~loss"]))
    assert cfg.parameter.seed == 11 and "loss" not in cfg


def test_run_dir_interpolation():
    now = datetime.datetime(2026, 1, 2, 3, 4, 5)
    full = compose(str(CONF_DIR), "config", ["parameter.seed=9"], now=now)
    assert full.hydra.run.dir == "results/cifar10/seed-9/2026-01-02/03-04-05"
    assert str(full.hydra.sweep.subdir) == "0"


def test_parse_value():
    assert parse_value("1e-4") == pytest.approx(1e-4)
    assert parse_value("true") is True
    assert parse_value("12") == 12
    assert parse_value("abc") == "abc"
    assert parse_value("[1, 2]") == [1, 2]
    assert parse_value("null") is None


def test_hydra_main_run_dir_and_multirun(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    seen = []

    @hydra_main(config_path=str(CONF_DIR), config_name="config")
    def app(cfg):
        import os
        seen.append((cfg.parameter.seed, os.getcwd()))
        return cfg.parameter.seed

    out = app([f"hydra.run.dir={tmp_path}/run", "parameter.seed=3"])
    assert out == 3 and seen[-1][1] == str(tmp_path / "run")
    assert (tmp_path / "run" / ".hydra" / "config.yaml").exists()
    assert (tmp_path / "run" / ".hydra" / "overrides.yaml").exists()
    res = app(["-m", f"hydra.sweep.dir={tmp_path}/sweep", "parameter.seed=1,2"])
    assert res == [1, 2]
    assert (tmp_path / "sweep" / "0").is_dir() and (tmp_path / "sweep" / "1").is_dir()
