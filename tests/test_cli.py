"""End-to-end CLI on CPU: pretrain → checkpoint (reference format) → eval results.json schema →
resume; supervised baseline keeps only the best checkpoint."""
import json
import subprocess
import sys
from pathlib import Path

import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
COMMON = ["data.synthetic=true", "data.synthetic_size=32", "experiment.batches=8",
          "experiment.base_cnn=resnet18"]


def _run(script, args, cwd):
    r = subprocess.run([sys.executable, str(ROOT / script), *args], cwd=str(cwd),
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout + r.stderr


@pytest.mark.timeout(900)
def test_pretrain_eval_resume(tmp_path):
    run = tmp_path / "run"
    out = _run("main.py", COMMON + ["parameter.epochs=2", "parameter.warmup_epochs=1",
                                    "experiment.save_model_epoch=1", f"hydra.run.dir={run}"],
               tmp_path)
    assert "Epoch:2/2 progress:1.000 loss:" in out
    ck = torch.load(run / "epoch=2-cifar10.pt", weights_only=True)
    assert len(ck) == 128 and all(k.startswith("module.") for k in ck)
    lines = [json.loads(l) for l in (run / "metrics.jsonl").read_text().splitlines()]
    assert lines[-1]["epoch"] == 2 and lines[-1]["images_per_sec"] > 0
    # resume from epoch 1 reproduces epoch 2's logged loss
    run2 = tmp_path / "run2"
    out2 = _run("main.py", COMMON + ["parameter.epochs=2", "parameter.warmup_epochs=1",
                                     "experiment.save_model_epoch=1", f"hydra.run.dir={run2}",
                                     f"runtime.resume={run / 'resume-1.pt'}"], tmp_path)
    l1 = [l for l in out.splitlines() if "Epoch:2/2" in l][0].split("loss:")[1]
    l2 = [l for l in out2.splitlines() if "Epoch:2/2" in l][0].split("loss:")[1]
    assert l1 == l2
    # eval: centroid and linear
    ev = tmp_path / "ev"
    _run("eval.py", ["data.synthetic=true", "data.synthetic_size=32", "experiment.batches=8",
                     f"experiment.target_dir={run}", f"hydra.run.dir={ev}"], tmp_path)
    res = json.loads((ev / "results.json").read_text())
    assert set(res) == {"epoch=1-cifar10.pt", "epoch=2-cifar10.pt"}
    assert set(res["epoch=2-cifar10.pt"]) == {"train_acc", "train_top_5_acc", "val_acc",
                                             "val_top_5_acc"}
    ev2 = tmp_path / "ev2"
    _run("eval.py", ["data.synthetic=true", "data.synthetic_size=32", "experiment.batches=8",
                     f"experiment.target_dir={run}", "parameter.classifier=linear",
                     "parameter.epochs=2", "parameter.use_full_encoder=true",
                     f"hydra.run.dir={ev2}"], tmp_path)
    r2 = json.loads((ev2 / "results.json").read_text())["epoch=1-cifar10.pt"]
    assert len(r2["val_accuracies"]) == 2 and "highest_val_top_k_acc" in r2


@pytest.mark.timeout(600)
def test_supervised_keeps_best_only(tmp_path):
    run = tmp_path / "sup"
    out = _run("supervised.py", COMMON + ["parameter.epochs=3", "parameter.warmup_epochs=1",
                                          f"hydra.run.dir={run}"], tmp_path)
    assert "val acc:" in out
    cks = list(run.glob("epoch=*-cifar10.pt"))
    assert len(cks) == 1
